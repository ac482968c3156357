# Round-4 run d: pass-B experiments, reverse queue sweep, config 2 profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_exp_b2.sh || exit 1
bash tools/gpu_exp_rev.sh || exit 2
bash tools/gpu_prof_cfg.sh || exit 3
echo R04DOK
