#!/bin/bash
# Round check on a GPU box: GPU tests, smoke, 1-GPU bench, kernel stats.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAIL rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "BENCH FAIL"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "PROF FAIL"; exit 1; }
  echo prof ok
fi
