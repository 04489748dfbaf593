#!/bin/bash
# One kernel-iteration check on a GPU box: the GPU tests selected by $TESTS (pytest -k expression; all GPU tests
# when empty), the default 1-GPU bench, and (PROF=1) rocprofv3 kernel stats of the bench.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
K=()
[ -n "$TESTS" ] && K=(-k "$TESTS")
timeout -k 10 900 python -u -m pytest tests -m gpu "${K[@]}" -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_iter.log 2>&1 || { echo "PYTEST FAIL"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_iter.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_iter.log
timeout -k 10 240 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_iter.log 2>&1 \
    || { echo "BENCH FAIL"; tail -20 gpurun_out/bench_iter.log; exit 1; }
tail -1 gpurun_out/bench_iter.log | cut -c1-220
if [ -n "$PROF" ]; then
  rm -rf /tmp/kprof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof -o k --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 ${BENCH_ARGS:-} > "$ROOT/gpurun_out/kprof.log" 2>&1) \
      || { echo "PROF FAIL"; tail -20 gpurun_out/kprof.log; exit 4; }
  f=$(find /tmp/kprof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kstats_iter.csv
  python3 scripts/prof_summary.py gpurun_out/kstats_iter.csv 7 "${PROF_TITLE:-iteration}" > gpurun_out/kstats_iter.md
  head -22 gpurun_out/kstats_iter.md | tail -17
fi
