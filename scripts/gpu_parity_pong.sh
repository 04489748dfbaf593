#!/bin/bash
# bf16 vs fp32 engine learning parity on Pong pixels (N=4, 16 paths x 16 envs, T=5; profiles/solve/learn_r2
# s16_mean_tn config).  SEEDS="1 2", BUDGET_BF16 / BUDGET_FP32 in seconds.  Records go to gpurun_out/parity/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/parity
export TMPDIR=/tmp
S="--paths 16 --envs 16 --tmax 5"
for d in bf16 fp32; do
  timeout -k 10 200 python -u bench.py $S --steps 20 --warmup 5 --dtype $d > gpurun_out/parity/bench_$d.log 2>&1 \
      || { echo "BENCH FAIL $d"; tail -20 gpurun_out/parity/bench_$d.log; exit 1; }
  echo "bench $d: $(tail -1 gpurun_out/parity/bench_$d.log | cut -c1-120)"
done
C="--preset pong --ga-backend device --report-every 30 --N 4 --fitness mean --trunk-scale none $S"
for seed in ${SEEDS:-1}; do
  for d in ${DTYPES:-fp32 bf16}; do
    b=$([ $d = fp32 ] && echo ${BUDGET_FP32:-420} || echo ${BUDGET_BF16:-240})
    name=pong_s16_${d}_seed$seed
    timeout -k 10 $((b + 150)) python -u scripts/solve.py $C --seed $seed --dtype $d --minutes $(python3 -c "print($b/60)") \
        --curve gpurun_out/parity/$name.jsonl --out gpurun_out/parity/$name.json > gpurun_out/parity/$name.log 2>&1 \
        || { echo "RUN FAIL $name"; tail -5 gpurun_out/parity/$name.log; exit 1; }
    echo "== $name: $(tail -1 gpurun_out/parity/$name.json | cut -c1-330)"
  done
done
