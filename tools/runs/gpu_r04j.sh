# Round-4 run j: pass A's hashed histogram (> 8192 bricks): parity (forced hash / overflow
# at small grids, the 1024^3 and 9216-brick config tests, long rays), then config 5's shard
# bench line and a kernel trace of its pipelined calls (does pass A now run beside F?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py > $O/tests.txt 2>&1 || { echo TESTFAIL; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 500 python3 bench.py --image 1280x720 --grid 1024 --poses-per-gpu 256 --steps 12 --warmup 2 --cpu-frames 0 --no-secondary --pmc off > $O/config5shard.json 2> $O/config5shard.err || { echo "FAIL cfg5"; tail -5 $O/config5shard.err; exit 2; }
python3 tools/show_bench.py $O/config5shard.json | head -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/exp_fuse.py --tag cfg5 --grid 1024 --image 1280x720 --poses 256 --calls 6 > $O/kt.json 2> $O/kt.err || { echo KTFAIL; tail -5 $O/kt.err; exit 3; }
cat $O/kt.json
echo R04JOK
