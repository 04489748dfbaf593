#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pathnet_gym_amd.cli supervised --tasks mnist,svhn --control > gpurun_out/supervised.json 2> gpurun_out/supervised.err || { tail -20 gpurun_out/supervised.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/supervised.json')); print({k: d[k] for k in ('generations_to_accuracy','seconds')}, [t['best_accuracy'] for t in d['per_task']], d['control']['best_accuracy'])"
for seed in 1 2 3; do
  timeout -k 10 400 python scripts/solve.py --preset pong --N 10 --paths 16 --envs 16 --tmax 5 --ga-backend device --seed $seed --minutes 5 --report-every 20 --curve gpurun_out/solve_dev_s$seed.jsonl > gpurun_out/solve_dev_s$seed.log 2>&1 || { tail -5 gpurun_out/solve_dev_s$seed.log; exit 4; }
  tail -1 gpurun_out/solve_dev_s$seed.log
done
