#!/bin/bash
# Controlled N=4 learning ablation on one GPU: one factor at a time,
# same seed, same wall budget.  Usage: SECS=150 SHAPE="--paths 16 --envs 16 --tmax 5" scripts/gpu_ablate.sh [arm ...]
# Arms are NAME=FLAGS pairs; default: the five-arm table below.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
SECS=${SECS:-150}
SHAPE=${SHAPE:---paths 16 --envs 16 --tmax 5 --N 4}
COMMON="--preset pong --ga-backend device --seed ${SEED:-1} --report-every 30 --keep-going"
if [ $# -eq 0 ]; then
  set -- "base=" "trunk_none=--trunk-scale none" "sum=--env-reduction sum" "same_path=--same-path" "lr2e-3=--lr 2e-3"
fi
for arm in "$@"; do
  name=${arm%%=*}; flags=${arm#*=}
  echo "== $name: $flags"
  timeout -k 10 $((SECS + 120)) python -u scripts/solve.py $COMMON $SHAPE --minutes $(python3 -c "print($SECS/60)") \
      $flags --curve gpurun_out/abl/$name.jsonl --out gpurun_out/abl/$name.json > gpurun_out/abl/$name.log 2>&1 \
      || { echo "ARM FAIL $name rc=$?"; tail -20 gpurun_out/abl/$name.log; exit 1; }
  tail -1 gpurun_out/abl/$name.log | cut -c1-400
done
