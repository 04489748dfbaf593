#!/bin/bash
# One stage of the config-5 suite at the bench shape (scripts/continual.py), resumable across GPU calls:
#   scripts/c5_stage.sh SEED STAGE SECONDS   STAGE = pong | rest | control
# pong: task 1 (Pong) of the sequence with a continuation checkpoint; rest: resume it for Breakout, SpaceInvaders,
# Alien and the evaluations; control: the from-scratch runs of tasks 2-4.  State between calls travels in c5_ck/
# (copied back from gpurun_out/r4/c5/ after each call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
seed=$1 stage=$2 secs=$3
OUT=gpurun_out/r4/c5
mkdir -p "$OUT"
common=(--preset atari4 --tasks Pong,Breakout,SpaceInvaders,Alien --paths 64 --envs 32 --tmax 20
        --frames 1.8e9,9e8,4e8,4e8 --stop-after-solve 3e7 --dtype fp32x --ring --seed "$seed" --report-every 30)
name=c5_s${seed}
case $stage in
  pong)
    timeout -k 10 "$secs" python -u scripts/continual.py "${common[@]}" --max-tasks 1 \
        --checkpoint "$OUT/${name}_ck.safetensors" --out "$OUT/$name.json" > "$OUT/${name}_pong.log" 2>&1 ;;
  rest)
    cp c5_ck/${name}_ck.safetensors* "$OUT/" && cp c5_ck/$name.json "$OUT/" || exit 3
    timeout -k 10 "$secs" python -u scripts/continual.py "${common[@]}" --resume \
        --checkpoint "$OUT/${name}_ck.safetensors" --out "$OUT/$name.json" > "$OUT/${name}_rest.log" 2>&1 ;;
  control)
    timeout -k 10 "$secs" python -u scripts/continual.py "${common[@]}" --control-only \
        --out "$OUT/${name}_control.json" > "$OUT/${name}_control.log" 2>&1 ;;
  *) echo "stage?"; exit 2 ;;
esac
rc=$?
grep -v '"run"' "$OUT/${name}_${stage}.log" | tail -6 | cut -c1-300
exit $rc
