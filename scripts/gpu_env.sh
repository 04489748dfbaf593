#!/bin/bash
# env kernel check: bit-exactness tests, micro-benchmark, ring/packed bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "pong_env or ring or gradient_matches_oracle" > gpurun_out/pytest_env.log 2>&1 \
    || { echo "PYTEST FAIL"; tail -30 gpurun_out/pytest_env.log; exit 1; }
tail -1 gpurun_out/pytest_env.log
timeout -k 10 120 python -u scripts/env_microbench.py || exit 1
timeout -k 10 200 python -u bench.py --ring > gpurun_out/b1.log 2>&1 || { tail gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log | cut -c1-220
timeout -k 10 200 python -u bench.py > gpurun_out/b2.log 2>&1 || { tail gpurun_out/b2.log; exit 1; }
tail -1 gpurun_out/b2.log | cut -c1-220
