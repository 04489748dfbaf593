#!/bin/bash
# GPU tests, then generations-to-solve on the EXACT bench config for the given seeds (stop at solve).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/solve
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit 1; fi
grep -E "FAILED|^E  " gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
grep -E "^layer" gpurun_out/pytest_gpu.log | head -3
fi
for seed in ${SEEDS:-2 3}; do
  NAME=pong_bench${DT:+_$DT}_seed$seed
  timeout -k 10 $((${SECS:-480} + 120)) python -u scripts/solve.py --preset pong --ga-backend device --seed $seed \
      ${DT:+--dtype $DT} --report-every 30 --minutes $(python3 -c "print(${SECS:-480}/60)") \
      --curve gpurun_out/solve/$NAME.jsonl --out gpurun_out/solve/$NAME.json \
      > gpurun_out/solve/$NAME.log 2>&1 || { echo "SOLVE FAIL seed $seed"; tail -5 gpurun_out/solve/$NAME.log; exit 1; }
  echo "== seed $seed"; tail -1 gpurun_out/solve/$NAME.json | cut -c1-330
done
