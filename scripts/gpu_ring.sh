#!/bin/bash
# Frame-ring check: targeted GPU tests, then ring vs packed bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "ring or gradient_matches_oracle or pong_env or engine_update" > gpurun_out/pytest_ring.log 2>&1 \
    || { echo "PYTEST FAIL"; tail -40 gpurun_out/pytest_ring.log; exit 1; }
tail -3 gpurun_out/pytest_ring.log
timeout -k 10 300 python -u bench.py --ring > gpurun_out/bench_ring.log 2>&1 || { echo "BENCH FAIL"; tail -20 gpurun_out/bench_ring.log; exit 1; }
tail -1 gpurun_out/bench_ring.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_packed.log 2>&1 || { echo "BENCH2 FAIL"; tail -20 gpurun_out/bench_packed.log; exit 1; }
tail -1 gpurun_out/bench_packed.log
