# Round-4 run p: reverse parity with the 64-item spatial queue, then a sweep around it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04p
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "reverse" tests/test_reference_driver.py > gpurun_out/r04p/tests.txt 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/r04p/tests.txt; exit 1; }
tail -2 gpurun_out/r04p/tests.txt
REV_LIBS="r64_4_16 r64_8_24 r64_16_16 r64_8_8" bash tools/gpu_exp_rev.sh || exit 2
echo R04POK
