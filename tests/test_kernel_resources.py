"""CPU: the gfx950 kernels' register budgets (hipcc cross-compiles here).  Every kernel of the
product keeps its state in registers: no scratch (private segment) and no spilled VGPRs.  A
select between struct fields or a per-axis constant indexed by a lane's axis can silently become
a dynamically indexed private array (one such change made pass B 15x slower in round 5), so the
code objects' metadata is checked at every CPU run.  The hot kernels' VGPR counts are pinned to
their occupancy bands."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "depth-map-fusion-utils_amd")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-fno-gpu-flush-denormals-to-zero", "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"),
         "--cuda-device-only", "-S"]


def _kernels(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, *FLAGS, "-o", str(out), src], check=True, capture_output=True, timeout=600)
    meta = out.read_text().split(".end_amdgpu_metadata")[0].split("amdhsa.kernels:")[-1]
    kernels = {}
    for block in re.split(r"\n  - ", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        if not name:
            continue
        val = {k: int(m.group(1)) for k in ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count",
                                            "sgpr_spill_count")
               if (m := re.search(r"\." + k + r":\s+(\d+)", block))}
        kernels[name.group(1)] = val
    return kernels


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.timeout(900)
@pytest.mark.parametrize("src", ["dmf_fuse.hip", "dmf_trace.hip", "dmf_core.hip", "dmf_ogrid.hip", "dmf_comm.hip"])
def test_no_scratch_no_spills(src, tmp_path):
    # the engine's own kernels (namespace dmf; rocPRIM's library kernels are not ours)
    ks = {n: v for n, v in _kernels(os.path.join(PKG, "csrc", src), tmp_path).items() if n.startswith("_ZN3dmf")}
    assert ks, "no kernels parsed"
    bad = {n: v for n, v in ks.items() if v.get("private_segment_fixed_size", 0) or v.get("vgpr_spill_count", 0)}
    assert not bad, f"kernels with scratch or VGPR spills: {bad}"
    if src == "dmf_fuse.hip":
        f = [v for n, v in ks.items() if "k_bk_fuse_s" in n]
        b = [v for n, v in ks.items() if "k_bk_pairsILb1" in n]
        assert f and all(v["vgpr_count"] <= 64 for v in f)   # phase F: LDS bounds it to 4 waves/SIMD anyway
        assert b and all(v["vgpr_count"] <= 128 for v in b)  # pass B: 4 waves per SIMD
    if src == "dmf_trace.hip":
        r = [v for n, v in ks.items() if "k_reverse_x" in n]
        assert r and all(v["vgpr_count"] <= 80 for v in r)   # reverseRayTraceFast: 6 waves per SIMD
