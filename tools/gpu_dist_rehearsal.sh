# N = 2 rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks share the GPU
# over gloo (torch all-reduce merge; RCCL needs one GPU per rank), a few steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dist
DMF_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-3} --warmup 1 > gpurun_out/dist/n2.json 2> gpurun_out/dist/n2.err || { echo DISTFAIL; tail -30 gpurun_out/dist/n2.err; exit 1; }
cat gpurun_out/dist/n2.json
echo ALLOK
