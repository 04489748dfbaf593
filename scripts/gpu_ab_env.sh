#!/bin/bash
# A/B bench over environment settings: ARMS="A=1 B=2|C=3" (arm 0 = defaults).  One bench per arm, 20 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra AR <<< "${ARMS:-}"
i=0
for arm in "" "${AR[@]}"; do
  env $arm timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab_$i.log 2>&1 \
    || { echo "BENCH FAIL [$arm]"; tail -20 gpurun_out/ab_$i.log; exit 1; }
  echo "arm $i [$arm]: $(tail -1 gpurun_out/ab_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  i=$((i+1))
done
