#!/bin/bash
# From-scratch controls of tasks 2-4 of the 4-task suite (same config and budgets as _gpu_s2i.sh), seed SEED.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/continual
S=${SEED:-2}
timeout -k 10 1100 python -u scripts/continual.py --tasks Pong,Breakout,SpaceInvaders,Alien --seed $S --control-only \
    --frames 260e6,150e6,150e6,150e6 --stop-after-solve 20e6 --report-every 20 --out gpurun_out/continual/atari4_cal_ctrl_s$S.json \
    > gpurun_out/continual/atari4_cal_ctrl_s$S.log 2>&1 \
    || { echo "CONTROL FAIL"; tail -20 gpurun_out/continual/atari4_cal_ctrl_s$S.log; exit 1; }
grep -v '"run"\|"eval"' gpurun_out/continual/atari4_cal_ctrl_s$S.log | tail -4 | cut -c1-300
