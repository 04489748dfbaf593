#!/bin/bash
# Long evidence runs, part 1: fp32x generations-to-solve seed 3 at exactly the bench config, then the reference's own
# network (L=4 + LSTM 256) on synthetic Alien -> Centipede with a from-scratch Centipede control, seed 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/solve gpurun_out/continual
NAME=pong_bench_fp32x_seed3
timeout -k 10 600 python -u scripts/solve.py --preset pong --ga-backend device --seed 3 --dtype fp32x --report-every 30 \
    --minutes 8 --curve gpurun_out/solve/$NAME.jsonl --out gpurun_out/solve/$NAME.json > gpurun_out/solve/$NAME.log 2>&1 \
    || { echo "SOLVE FAIL"; tail -5 gpurun_out/solve/$NAME.log; exit 1; }
tail -1 gpurun_out/solve/$NAME.json | cut -c1-300
SEEDS=${SEEDS:-1} FRAMES=${FRAMES:-300e6,200e6} CAP=${CAP:-520} bash scripts/gpu_ref_lstm.sh
