#!/bin/bash
# From-scratch Breakout controls for the Pong -> Breakout continual run (same config, seeds 1 and 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/continual
for seed in 1 2; do
  timeout -k 10 540 python -u scripts/continual.py --tasks Pong,Breakout --control-only --seed $seed \
      --frames 300e6,200e6 --paths 16 --envs 16 --tmax 5 --report-every 20 \
      --out gpurun_out/continual/control_breakout_seed$seed.json > gpurun_out/continual/control_breakout_seed$seed.log 2>&1 \
    || { echo "CONTROL FAIL $seed"; tail -5 gpurun_out/continual/control_breakout_seed$seed.log; exit 1; }
  grep -v '"run"' gpurun_out/continual/control_breakout_seed$seed.log | tail -2 | cut -c1-400
done
