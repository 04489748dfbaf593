#!/bin/bash
# Generations-to-solve runs on one MI355X: CartPole-v1 (BASELINE config 2) then Pong (headline).
set -o pipefail
mkdir -p gpurun_out
PONG_MIN=${PONG_MIN:-13}
timeout -k 10 300 python scripts/solve.py --preset cartpole --minutes 3 --report-every 15 \
  --curve gpurun_out/solve_cartpole.jsonl > gpurun_out/solve_cartpole.log 2>&1 || { tail -30 gpurun_out/solve_cartpole.log; exit 1; }
tail -1 gpurun_out/solve_cartpole.log
timeout -k 10 $((PONG_MIN*60+180)) python scripts/solve.py --preset pong --minutes $PONG_MIN --report-every 30 \
  --curve gpurun_out/solve_pong.jsonl $PONG_ARGS > gpurun_out/solve_pong.log 2>&1 || { tail -30 gpurun_out/solve_pong.log; exit 1; }
tail -3 gpurun_out/solve_pong.log
