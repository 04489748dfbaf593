#!/bin/bash
# The 8-GPU population (512 paths x 32 envs, the P_total of 8 ranks of the bench config) on ONE GPU: the same
# replicated GA, concurrent tournaments 4 (per-rank rule) vs 32 (scaled with P_total).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/solve
C=${C:-4}; seed=${SEED:-1}; DT=${DT:-fp32x}
NAME=pop512_c${C}${TAGX:-}_${DT}_seed$seed
timeout -k 10 $((${SECS:-1020} + 90)) python -u scripts/solve.py --preset pong --paths 512 --envs 32 --concurrent $C \
    --ga-backend device --seed $seed --dtype $DT --report-every 30 ${EXTRA:-} --minutes $(python3 -c "print(${SECS:-1020}/60)") \
    --curve gpurun_out/solve/$NAME.jsonl --out gpurun_out/solve/$NAME.json > gpurun_out/solve/$NAME.log 2>&1 \
    || { echo "SOLVE FAIL"; tail -5 gpurun_out/solve/$NAME.log; exit 1; }
tail -1 gpurun_out/solve/$NAME.json | cut -c1-400
