#!/bin/bash
# Continual 4-task sequence Pong -> Breakout -> SpaceInvaders -> Alien (BASELINE config 5 on ONE GPU; atari4
# preset, HIP game logic, per-task heads, frozen winner paths).  No scratch controls in this job (time limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/continual
TAG=${1:-atari4_seq}
shift
timeout -k 10 1130 python -u scripts/continual.py --tasks Pong,Breakout,SpaceInvaders,Alien \
    --out gpurun_out/continual/$TAG.json "$@" > gpurun_out/continual/$TAG.log 2>&1 \
    || { echo "CONTINUAL FAIL"; tail -20 gpurun_out/continual/$TAG.log; exit 1; }
grep -v '"run"' gpurun_out/continual/$TAG.log | tail -12
