#!/bin/bash
# The 8-GPU population (512 paths x 32 envs = 8 ranks of the bench config) on ONE GPU with today's per-rank
# concurrency rule: 4 concurrent tournaments for P_total = 512 (bf16 engine for throughput; same GA).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
C=4 SEED=1 DT=bf16 SECS=900 bash scripts/gpu_pop512.sh
