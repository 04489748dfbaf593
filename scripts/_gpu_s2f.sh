#!/bin/bash
# Long evidence runs, part 4: the 8-GPU population with concurrency scaled with P_total (32 concurrent tournaments).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
C=32 SEED=1 DT=bf16 SECS=960 bash scripts/gpu_pop512.sh
