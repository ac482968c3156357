# Round-4 run f: fusion parity after the int32 quantisation (incl. non-finite poses), pass-A
# cost serial / pipelined, config-2 part size sweep, reverse queue sweep around 256 items.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fuse" tests/test_gpu_pipeline.py > $OUT/tests.txt 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
for mode in serial pipelined; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$mode -o run -- python3 tools/exp_fuse.py --tag a32_$mode --calls 20 --modes $mode > $OUT/a32_$mode.json 2> $OUT/a32_$mode.err || { echo "FAIL $mode"; tail -5 $OUT/a32_$mode.err; exit 2; }
  cat $OUT/a32_$mode.json
  python3 tools/kt_timeline.py $OUT/kt_$mode > $OUT/timeline_$mode.txt 2>&1; tail -11 $OUT/timeline_$mode.txt
done
for k in part_max=65535 part_max=49152 part_max=32768 tail_split=1; do
  timeout -k 10 200 python3 tools/exp_fuse.py --tag cfg2_$k --grid 256 --poses 64 --calls 60 --modes pipelined --knob $k > $OUT/cfg2_$k.json 2> $OUT/cfg2_$k.err || { echo "FAIL $k"; tail -5 $OUT/cfg2_$k.err; exit 3; }
  cat $OUT/cfg2_$k.json
done
REV_LIBS="r256_8_16 r128_8_16 r256_4_16 r256_8_32 r256_16_16" bash tools/gpu_exp_rev.sh || exit 4
echo R04FOK
