"""CPU self-tests of the exact arithmetic the kernels rely on (no GPU):
* tools/brick_selftest.cpp — the brick decomposition of the fusion DDA (dmf_brick.hpp)
  restarts the fine walk on exactly the cells the plain walk visits in each brick;
* tools/fastdiv_selftest.cpp — div_rn (dmf_internal.hpp) equals IEEE division over the
  projection and reverse-march domains."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_and_run(src, out, args, extra=()):
    exe = os.path.join(out, os.path.basename(src)[:-4])
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *extra, src, "-o", exe], check=True)
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)


def test_brick_decomposition_selftest(tmp_path):
    r = _build_and_run(os.path.join(ROOT, "tools", "brick_selftest.cpp"), str(tmp_path), ["100000", "3"],
                       ["-I", os.path.join(ROOT, "depth-map-fusion-utils_amd", "csrc")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failures" in r.stdout


@pytest.mark.timeout(300)
def test_fast_division_selftest(tmp_path):
    r = _build_and_run(os.path.join(ROOT, "tools", "fastdiv_selftest.cpp"), str(tmp_path), [])
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
