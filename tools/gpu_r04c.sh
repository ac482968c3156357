# Round-4 run c: pass-B diagnostics, then config 2's timeline + PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_exp_b2.sh || exit 1
bash tools/gpu_prof_cfg.sh || exit 2
echo R04COK
