#!/bin/bash
# Round check (GPU tests, smoke, bench) followed by the N=4 ablation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_round.sh && bash scripts/gpu_ablate.sh "$@"
