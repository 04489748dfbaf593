# two generations-to-solve seeds of the bench config at once on one GPU (scripts/solve.py, v2 criterion,
# deterministic fp32x): bash scripts/diag/cmd_r6_seeds.sh SEED_A SEED_B [MINUTES]
set -o pipefail
OUT=gpurun_out/r6/solve
mkdir -p $OUT
MIN=${3:-17.5}
S="--preset pong --paths 64 --envs 32 --ring --dtype fp32x --ga-backend device --deterministic --report-every 30"
pids=()
for seed in $1 $2; do
  # "1r": a repeat of seed 1 under its own name (the deterministic mode must reproduce it exactly)
  timeout -k 10 $(python3 -c "print(int($MIN*60+90))") python -u scripts/solve.py --minutes $MIN $S --seed ${seed%r} \
      --curve $OUT/v2_seed$seed.jsonl --out $OUT/v2_seed$seed.json > $OUT/v2_seed$seed.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
for seed in $1 $2; do
  tail -1 $OUT/v2_seed$seed.json 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seed $seed', d['stopped'], d['solved'], d['generations_to_solve'], d['updates_to_solve'], d.get('heldout_mean'), d.get('lr_at_solve'), d['updates_run'], d['wall_s'], len(d['candidates']))" || { echo "seed $seed: no record"; tail -5 $OUT/v2_seed$seed.log; }
done
exit $rc
