#!/bin/bash
# Round 6: rehearsal of the driver's 8-rank launch on a one-GPU box:
# `python bench.py --gpus 8` with NO wrapper (bench.py starts its 8 ranks itself), the ranks
# sharing the GPU over gloo (RCCL needs one GPU per rank), 8 poses per rank at 128^3: the 64-pose
# global set's digest is committed (tests/golden/fusion_digests.json[rehearsal_g128_N8]), so the
# line must print digest_match true.  Then N = 1 over the same 64 poses (same digest).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_dist
mkdir -p $O
DMF_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 8 --grid 128 --poses-per-gpu 8 --steps 50 --warmup 2 > $O/bench_n8_gloo_selflaunch.json 2> $O/bench_n8.err || { echo N8FAIL; tail -30 $O/bench_n8.err; exit 1; }
timeout -k 10 300 python3 bench.py --grid 128 --poses-per-gpu 64 --steps 50 --warmup 2 --pmc off --no-secondary --cpu-frames 0 --cpu-reverse-poses 0 > $O/bench_n1_64poses.json 2> $O/bench_n1.err || { echo N1FAIL; tail -30 $O/bench_n1.err; exit 2; }
python3 - <<'PY' || exit 3
import json
a = json.load(open("gpurun_out/r06_dist/bench_n8_gloo_selflaunch.json")); b = json.load(open("gpurun_out/r06_dist/bench_n1_64poses.json"))
print("N=8 gloo", a["n_gpus"], a["config"]["global_poses"], a["logodds_digest"], a["digest_match"], a["rccl"], "| N=1", b["logodds_digest"], b["digest_match"])
assert a["n_gpus"] == 8 and a["digest_match"] is True and b["digest_match"] is True
assert a["logodds_digest"] == b["logodds_digest"]
print("DIGESTS EQUAL")
PY
echo ALLOK
