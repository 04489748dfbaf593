#!/bin/bash
# The 8-GPU population on one GPU, concurrency scaled with P_total (32 tournaments), gradient summed over all paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
C=32 SEED=1 DT=bf16 SECS=900 bash scripts/gpu_pop512.sh
