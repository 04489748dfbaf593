#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 5; }
csv=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py "$csv" 7 "Pong PathNet update kernel stats" > gpurun_out/prof_summary.md && head -30 gpurun_out/prof_summary.md
exit $rc
