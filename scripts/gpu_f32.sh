#!/bin/bash
# fp32 engine mode + deterministic switch: GPU tests, then fp32 / deterministic / default bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_f32_engine.py -x -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_f32.log 2>&1 || { echo "PYTEST FAIL"; grep -E "PASS|FAIL|Error|^E " gpurun_out/pytest_f32.log | tail -40; exit 1; }
grep -E "PASS|per layer" gpurun_out/pytest_f32.log | cut -c1-300
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 10 --warmup 3 > gpurun_out/bench_fp32.log 2>&1 || { echo "BENCH FP32 FAIL"; tail -20 gpurun_out/bench_fp32.log; exit 1; }
tail -1 gpurun_out/bench_fp32.log | cut -c1-400
timeout -k 10 300 python -u bench.py --deterministic --steps 10 --warmup 3 > gpurun_out/bench_det.log 2>&1 || { echo "BENCH DET FAIL"; tail -20 gpurun_out/bench_det.log; exit 1; }
tail -1 gpurun_out/bench_det.log | cut -c1-400
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof32" -o f32 --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --dtype fp32 --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof32.log" 2>&1 || { echo "PROF FAIL"; exit 1; }
  echo prof ok
fi
