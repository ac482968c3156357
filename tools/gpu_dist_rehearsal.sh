# N = 2 rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks share the GPU
# over gloo (torch all-reduce merge + slab finalize on the comm lane; RCCL needs one GPU per
# rank), then N = 1 over the same global poses: the merged log-odds digests must be equal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dist
PL=${PL:-16}
DMF_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --poses-per-gpu $PL --steps ${STEPS:-3} --warmup 1 --pmc off --no-secondary --cpu-frames 0 > gpurun_out/dist/n2.json 2> gpurun_out/dist/n2.err || { echo DISTFAIL; tail -30 gpurun_out/dist/n2.err; exit 1; }
timeout -k 10 300 python bench.py --poses-per-gpu $((2 * PL)) --steps ${STEPS:-3} --warmup 1 --pmc off --no-secondary --cpu-frames 0 --cpu-reverse-poses 0 > gpurun_out/dist/n1.json 2> gpurun_out/dist/n1.err || { echo N1FAIL; tail -30 gpurun_out/dist/n1.err; exit 2; }
python3 - <<'PY' || exit 3
import json
a = json.load(open("gpurun_out/dist/n2.json")); b = json.load(open("gpurun_out/dist/n1.json"))
print("N=2 gloo", a["logodds_digest"], a["step_breakdown_ms"]["merge_kind"], "| N=1", b["logodds_digest"])
assert a["logodds_digest"] == b["logodds_digest"], "merged log-odds differ from one rank fusing all poses"
print("DIGESTS EQUAL")
PY
echo ALLOK
