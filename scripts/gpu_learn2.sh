#!/bin/bash
# GPU tests + bench + the headline config (64 paths x 32 envs, T=20, N=4) learning with trunk scale none
# and the windowed-mean GA fitness.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/learn2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit 1; fi
grep -E "FAILED|^E  " gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
grep -E "^\{" gpurun_out/pytest_gpu.log | head -5
C="--preset pong --ga-backend device --seed 1 --report-every 30 --keep-going --N 4 --fitness mean --trunk-scale none"
run() { name=$1; secs=$2; shift 2
  timeout -k 10 $((secs + 120)) python -u scripts/solve.py $C --minutes $(python3 -c "print($secs/60)") "$@" \
      --curve gpurun_out/learn2/$name.jsonl --out gpurun_out/learn2/$name.json > gpurun_out/learn2/$name.log 2>&1 \
      || { echo "RUN FAIL $name"; tail -5 gpurun_out/learn2/$name.log; exit 1; }
  echo "== $name"; tail -3 gpurun_out/learn2/$name.jsonl | cut -c1-250; tail -1 gpurun_out/learn2/$name.json | cut -c1-200; }
run bench_tn_mean 420 --paths 64 --envs 32 --tmax 20
