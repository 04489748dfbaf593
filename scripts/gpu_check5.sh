#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 5; }
csv=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py "$csv" 7 "Pong PathNet update kernel stats" > gpurun_out/prof_summary.md && head -24 gpurun_out/prof_summary.md
SWEEP_FILE=scripts/sweep_configs4.txt SWEEP_MIN=4 bash scripts/gpu_sweep.sh
