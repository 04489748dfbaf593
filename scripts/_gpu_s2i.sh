#!/bin/bash
# 4-task continual suite Pong -> Breakout -> SpaceInvaders -> Alien (atari4 preset, 16 paths x 16 envs, T=5, bf16,
# calibrated thresholds), one sequence seed (SEED), budgets 260 M / 150 M / 150 M / 150 M frames, each task ending 20 M frames after it solves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/continual
S=${SEED:-2}
timeout -k 10 1100 python -u scripts/continual.py --tasks Pong,Breakout,SpaceInvaders,Alien --seed $S \
    --frames 260e6,150e6,150e6,150e6 --stop-after-solve 20e6 --report-every 20 --out gpurun_out/continual/atari4_cal_seq_s$S.json \
    > gpurun_out/continual/atari4_cal_seq_s$S.log 2>&1 \
    || { echo "SEQUENCE FAIL"; tail -20 gpurun_out/continual/atari4_cal_seq_s$S.log; exit 1; }
grep -v '"run"\|"eval"' gpurun_out/continual/atari4_cal_seq_s$S.log | tail -6 | cut -c1-300
