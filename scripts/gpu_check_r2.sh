#!/bin/bash
# Full GPU test suite, counter diagnostic without the fence, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAIL"; grep -E "PASS|FAIL|Error|^E " gpurun_out/pytest_gpu.log | tail -40; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 150 python -u scripts/diag_pipeline3.py 20000 nofence > gpurun_out/diag5_nofence.log 2>&1 || { echo "DIAG FAIL"; tail -5 gpurun_out/diag5_nofence.log; exit 1; }
tail -1 gpurun_out/diag5_nofence.log | cut -c1-600
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r2a.log 2>&1 || { echo "BENCH FAIL"; tail -20 gpurun_out/bench_r2a.log; exit 1; }
tail -1 gpurun_out/bench_r2a.log | cut -c1-700
