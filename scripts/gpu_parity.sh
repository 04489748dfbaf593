#!/bin/bash
# bf16 HIP engine vs fp32 torch backend: generations-to-solve on CartPole-v1 (BASELINE config 2 shape), 5 seeds each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/parity
for seed in 1 2 3 4 5; do
  for be in hip torch; do
    timeout -k 10 200 python -u scripts/solve.py --preset cartpole --backend $be --seed $seed --minutes 2.5 \
        --report-every 10 --curve gpurun_out/parity/cartpole_${be}_seed$seed.jsonl \
        --out gpurun_out/parity/cartpole_${be}_seed$seed.json > gpurun_out/parity/cartpole_${be}_seed$seed.log 2>&1 \
      || { echo "RUN FAIL $be $seed"; tail -5 gpurun_out/parity/cartpole_${be}_seed$seed.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['solved'], d['generations_to_solve'], d['frames_to_solve'], d['seconds'], d['config']['dtype'])" gpurun_out/parity/cartpole_${be}_seed$seed.json
  done
done
