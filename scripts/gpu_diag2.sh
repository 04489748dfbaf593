#!/bin/bash
# Bridge GPU tests + pipelined-counter diagnostic (graph and eager).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gym_bridge.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_bridge.log 2>&1 || { echo "BRIDGE TESTS FAIL"; tail -30 gpurun_out/pytest_bridge.log; exit 1; }
tail -3 gpurun_out/pytest_bridge.log
timeout -k 10 150 python -u scripts/diag_pipeline.py 60 graph > gpurun_out/diag_graph.log 2>&1 || { echo "DIAG FAIL"; tail -20 gpurun_out/diag_graph.log; exit 1; }
tail -14 gpurun_out/diag_graph.log | cut -c1-600
timeout -k 10 150 python -u scripts/diag_pipeline.py 45 nograph > gpurun_out/diag_nograph.log 2>&1 || { echo "DIAG2 FAIL"; tail -20 gpurun_out/diag_nograph.log; exit 1; }
tail -14 gpurun_out/diag_nograph.log | cut -c1-600
