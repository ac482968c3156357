# reverseRayTraceFast work-queue lane occupancy (DMF_EXP_STATS build): spatial order
# (knob 0, the default 128/8/16 queue) vs insertion order (knob 3, 512/8/8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rev_stats
mkdir -p $OUT
DMF_LIB=depth-map-fusion-utils_amd/build_exp/rstats/libdmf.so timeout -k 10 200 python3 tools/exp_reverse.py > $OUT/rstats.json 2> $OUT/rstats.err || { echo FAIL; tail -5 $OUT/rstats.err; exit 1; }
cat $OUT/rstats.json
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_pipeline.py > $OUT/pipeline_tests.txt 2>&1 || { echo TESTFAIL; tail -20 $OUT/pipeline_tests.txt; exit 2; }
tail -2 $OUT/pipeline_tests.txt
echo REVSTATSOK
