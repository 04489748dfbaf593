#!/bin/bash
# Learning ablation, several arms at once on one GPU (small latency-bound configs share it well).
# Usage: SECS=150 PAR=3 scripts/gpu_ablate_par.sh "name=flags" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abl2
export TMPDIR=/tmp
SECS=${SECS:-150}
PAR=${PAR:-3}
SHAPE=${SHAPE:---paths 16 --envs 16 --tmax 5 --N 4}
COMMON="--preset pong --ga-backend device --seed ${SEED:-1} --report-every 30 --keep-going"
MIN=$(python3 -c "print($SECS/60)")
run_batch() {
  local pids=()
  for arm in "$@"; do
    name=${arm%%=*}; flags=${arm#*=}
    timeout -k 10 $((SECS + 150)) python -u scripts/solve.py $COMMON $SHAPE --minutes $MIN $flags \
        --curve gpurun_out/abl2/$name.jsonl --out gpurun_out/abl2/$name.json > gpurun_out/abl2/$name.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=1; done
  for arm in "$@"; do name=${arm%%=*}; echo "== $name"; tail -1 gpurun_out/abl2/$name.jsonl | cut -c1-220; done
  return $rc
}
batch=()
for arm in "$@"; do
  batch+=("$arm")
  if [ ${#batch[@]} -ge $PAR ]; then run_batch "${batch[@]}" || { echo "BATCH FAIL"; exit 1; }; batch=(); fi
done
if [ ${#batch[@]} -gt 0 ]; then run_batch "${batch[@]}" || { echo "BATCH FAIL"; exit 1; }; fi
