#!/bin/bash
# Perf iteration on one GPU: kernel tests, bench, rocprofv3 kernel stats.  Usage: gpu_perf.sh TAG [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
TAG=${1:-perf}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "$K" \
      > gpurun_out/test_$TAG.log 2>&1 || { echo "TEST FAIL"; tail -30 gpurun_out/test_$TAG.log; exit 1; }
  tail -2 gpurun_out/test_$TAG.log
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { echo "BENCH FAIL"; tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-220
rm -rf /tmp/kprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof -o k --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 ${BENCH_ARGS:-} > "$ROOT/gpurun_out/kprof_$TAG.log" 2>&1) || { echo "PROF FAIL"; tail -20 gpurun_out/kprof_$TAG.log; exit 1; }
f=$(find /tmp/kprof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kstats_$TAG.csv
python3 scripts/prof_summary.py gpurun_out/kstats_$TAG.csv 13 "$TAG" > gpurun_out/kstats_$TAG.md
head -24 gpurun_out/kstats_$TAG.md
