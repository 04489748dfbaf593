#!/bin/bash
# Pong learnability sweep (HIP engine, 1 GPU): each config runs SWEEP_MIN minutes.
mkdir -p gpurun_out
MIN=${SWEEP_MIN:-3}
i=0
while IFS= read -r cfg; do
  [ -z "$cfg" ] && continue
  i=$((i+1))
  echo "== sweep $i: $cfg"
  timeout -k 10 $((MIN*60+150)) python scripts/solve.py --preset pong --minutes $MIN --report-every 20 \
    --curve gpurun_out/sweep_$i.jsonl $cfg > gpurun_out/sweep_$i.log 2>&1
  rc=$?
  tail -1 gpurun_out/sweep_$i.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/sweep_$i.log; exit $rc; fi
done < "${SWEEP_FILE:-scripts/sweep_configs.txt}"
