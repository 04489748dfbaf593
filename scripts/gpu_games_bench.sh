#!/bin/bash
# Throughput of every synthetic game on the atari4 preset (18-way head) with the HIP game logic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/games
for g in Pong Breakout SpaceInvaders Alien MsPacman Centipede; do
  timeout -k 10 240 python -u bench.py --preset atari4 --env $g --steps 10 --warmup 3 > gpurun_out/games/bench_$g.log 2>&1 \
    || { echo "BENCH FAIL $g"; tail -5 gpurun_out/games/bench_$g.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/games/bench_$g.log $g
done
