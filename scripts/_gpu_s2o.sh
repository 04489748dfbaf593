#!/bin/bash
# fp32x generations-to-solve, seed 3, exactly the bench config, 16-minute budget (the first seed-3 run was cut at
# 480 s unsolved); the record replaces profiles/solve/pong_bench_fp32x_seed3.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/solve
NAME=pong_bench_fp32x_seed3
timeout -k 10 1050 python -u scripts/solve.py --preset pong --ga-backend device --seed 3 --dtype fp32x --ring --report-every 30 \
    --minutes 16 --curve gpurun_out/solve/$NAME.jsonl --out gpurun_out/solve/$NAME.json > gpurun_out/solve/$NAME.log 2>&1 \
    || { echo "SOLVE FAIL"; tail -5 gpurun_out/solve/$NAME.log; exit 1; }
tail -1 gpurun_out/solve/$NAME.json | cut -c1-300
