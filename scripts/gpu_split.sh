#!/bin/bash
# Split-rollout check on a GPU box: bit-identity tests, bench A/B (1 vs 2 vs 4 path groups), full GPU suite,
# kernel stats of the default bench.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_split_rollout.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_split.log 2>&1 || { echo "SPLIT TEST FAIL"; tail -40 gpurun_out/pytest_split.log; exit 1; }
tail -3 gpurun_out/pytest_split.log
for g in ${BENCH_GROUPS:-1 2 4}; do
  timeout -k 10 240 python -u bench.py --rollout-groups $g > gpurun_out/bench_g$g.log 2>&1 \
      || { echo "BENCH FAIL g=$g"; tail -20 gpurun_out/bench_g$g.log; exit 1; }
  echo "g=$g $(tail -1 gpurun_out/bench_g$g.log | cut -c1-200)"
done
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAIL"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { echo "SMOKE FAIL"; tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [ -n "$PROF" ]; then
  rm -rf /tmp/kprof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof -o k --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/kprof.log" 2>&1) \
      || { echo "PROF FAIL"; tail -20 gpurun_out/kprof.log; exit 4; }
  f=$(find /tmp/kprof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kstats_split.csv
  python3 scripts/prof_summary.py gpurun_out/kstats_split.csv 7 "split rollout" > gpurun_out/kstats_split.md
  head -30 gpurun_out/kstats_split.md
fi
