#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/runs/gpu_r05c.sh && bash tools/runs/gpu_r05d.sh
