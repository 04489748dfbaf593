#!/bin/bash
# A/B of kernel switches on the headline bench (1 GPU).  Usage: OPTS="a=1;b=2|c=3" scripts/gpu_ab.sh
# ('|' separates arms, ';' separates switches inside one arm; the empty arm = defaults).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "$TESTS" \
      > gpurun_out/pytest_ab.log 2>&1 || { echo "PYTEST FAIL"; tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -1 gpurun_out/pytest_ab.log
fi
IFS='|' read -ra ARMS <<< "${OPTS:-}"
[ ${#ARMS[@]} -eq 0 ] && ARMS=("")
for arm in "" "${ARMS[@]}"; do
  args=""
  IFS=';' read -ra KV <<< "$arm"
  for kv in "${KV[@]}"; do [ -n "$kv" ] && args="$args --kernel-opt $kv"; done
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 $args > gpurun_out/ab.log 2>&1 || { echo "BENCH FAIL [$arm]"; tail -20 gpurun_out/ab.log; exit 4; }
  echo "[$arm] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
