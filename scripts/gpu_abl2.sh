#!/bin/bash
# Graph-fence regression test + bench + the N=4 ablation again (round-1 device-GA runs raced).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_pipeline.py -m gpu -x -v --timeout 150 --timeout-method thread \
    > gpurun_out/pytest_pipeline.log 2>&1 || { echo "PIPELINE TEST FAIL"; tail -30 gpurun_out/pytest_pipeline.log; exit 1; }
tail -2 gpurun_out/pytest_pipeline.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_fence.log 2>&1 || { echo "BENCH FAIL"; tail -20 gpurun_out/bench_fence.log; exit 1; }
tail -1 gpurun_out/bench_fence.log | cut -c1-400
SECS=${SECS:-140} bash scripts/gpu_ablate.sh "base=" "trunk_none=--trunk-scale none" "sum=--env-reduction sum" \
    "same_path=--same-path" "lr2e-3=--lr 2e-3" "n10_control=--N 10"
