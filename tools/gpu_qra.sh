set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
DMF_LIB=depth-map-fusion-utils_amd/build_exp/qra/libdmf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 180 --timeout-method thread -k "fuse or config" > gpurun_out/qra_tests.log 2>&1 || { echo QRATESTFAIL; tail -30 gpurun_out/qra_tests.log; exit 1; }
tail -2 gpurun_out/qra_tests.log
EXPS="base qra base qra" timeout -k 10 500 bash tools/gpu_exp_libs.sh || exit 2
bash tools/profile_round.sh r02 || exit 3
echo DONE
