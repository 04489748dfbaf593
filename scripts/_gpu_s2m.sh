#!/bin/bash
# The 8-GPU population with the concurrency scaled with P_total: 32 concurrent tournaments (= paths / 16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
C=32 SEED=1 DT=bf16 SECS=900 bash scripts/gpu_pop512.sh
