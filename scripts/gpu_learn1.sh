#!/bin/bash
# GPU tests + bench + N=4 learning with the windowed-mean GA fitness (window = envs per path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/learn1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
# assertion failures (rc 1) are reported and the learning runs still go; anything else (crash, timeout) stops here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit 1; fi
grep -E "FAILED|^E " gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_f16.log 2>&1 || { echo "BENCH FAIL"; tail -20 gpurun_out/bench_f16.log; exit 1; }
tail -1 gpurun_out/bench_f16.log | cut -c1-300
C="--preset pong --ga-backend device --seed 1 --report-every 30 --keep-going --N 4 --fitness mean"
run() { name=$1; secs=$2; shift 2
  timeout -k 10 $((secs + 120)) python -u scripts/solve.py $C --minutes $(python3 -c "print($secs/60)") "$@" \
      --curve gpurun_out/learn1/$name.jsonl --out gpurun_out/learn1/$name.json > gpurun_out/learn1/$name.log 2>&1 \
      || { echo "RUN FAIL $name"; tail -5 gpurun_out/learn1/$name.log; exit 1; }
  echo "== $name"; tail -2 gpurun_out/learn1/$name.jsonl | cut -c1-250; tail -1 gpurun_out/learn1/$name.json | cut -c1-200; }
run s16_mean 130 --paths 16 --envs 16 --tmax 5
run s16_mean_tn 130 --paths 16 --envs 16 --tmax 5 --trunk-scale none
run bench_mean 300 --paths 64 --envs 32 --tmax 20
