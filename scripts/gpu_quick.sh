#!/bin/bash
# kernel-change check: conv/fc numerics tests, bench, kernel stats.  TAG=name
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${TESTS:-trunk or fast_conv or slab or pipeline_variants or gradient_matches_oracle or fc_}" > gpurun_out/pytest_q.log 2>&1 \
    || { echo "PYTEST FAIL"; tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
timeout -k 10 200 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bq.log 2>&1 || { tail gpurun_out/bq.log; exit 1; }
tail -1 gpurun_out/bq.log | cut -c1-200
TAG=${TAG:-q} bash scripts/gpu_prof1.sh
