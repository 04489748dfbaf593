#!/bin/bash
# Continual Pong -> Breakout (atari4 preset, HIP game logic) with a scratch Breakout control.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/continual
TAG=${1:-pong_breakout}
shift
timeout -k 10 1100 python -u scripts/continual.py --tasks Pong,Breakout --control --out gpurun_out/continual/$TAG.json "$@" \
    > gpurun_out/continual/$TAG.log 2>&1 || { echo "CONTINUAL FAIL"; tail -20 gpurun_out/continual/$TAG.log; exit 1; }
grep -v '"run"' gpurun_out/continual/$TAG.log | tail -12
