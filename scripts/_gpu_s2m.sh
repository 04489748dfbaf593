#!/bin/bash
# The 8-GPU population on one GPU, concurrency scaled with P_total (32 tournaments) AND the gradient at the 1-GPU
# scale (x 1/8 = the all-reduced gradient of 8 ranks averaged, a2c.rank_reduction = "mean").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
C=32 SEED=1 DT=bf16 SECS=900 TAGX=_gs8 EXTRA="--grad-scale 0.125" bash scripts/gpu_pop512.sh
