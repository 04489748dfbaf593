#!/bin/bash
# Long evidence runs, part 3: supervised seed 3, then the 8-GPU population (512 paths x 32 envs) on one GPU with
# today's per-rank concurrency rule (4 concurrent tournaments for P_total = 512).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/_gpu_sup.sh 3 || exit 1
C=4 SEED=1 DT=bf16 SECS=840 bash scripts/gpu_pop512.sh
