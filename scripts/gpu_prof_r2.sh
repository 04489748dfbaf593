#!/bin/bash
# Kernel-time profile of the bench (rocprofv3 --kernel-trace --stats) + packed vs frame-ring bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench_packed.log 2>&1 || { echo "BENCH FAIL"; tail -5 gpurun_out/bench_packed.log; exit 1; }
tail -1 gpurun_out/bench_packed.log | cut -c1-200
timeout -k 10 300 python -u bench.py --ring > gpurun_out/bench_ring.log 2>&1 || { echo "BENCH RING FAIL"; tail -5 gpurun_out/bench_ring.log; exit 1; }
tail -1 gpurun_out/bench_ring.log | cut -c1-200
rm -rf /tmp/kprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof -o k --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 > "$ROOT/gpurun_out/kprof.log" 2>&1) || { echo "PROF FAIL"; tail -20 gpurun_out/kprof.log; exit 1; }
f=$(find /tmp/kprof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kstats_r2.csv
python3 scripts/prof_summary.py gpurun_out/kstats_r2.csv 13 "r2 fp16-offset conv1" > gpurun_out/kstats_r2.md
head -30 gpurun_out/kstats_r2.md
