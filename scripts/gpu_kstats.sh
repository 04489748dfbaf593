#!/bin/bash
# rocprofv3 kernel stats of the bench for one or more kernel-switch arms.  Usage: OPTS="a=1|b=2" scripts/gpu_kstats.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra ARMS <<< "${OPTS:-}"
i=0
for arm in "" "${ARMS[@]}"; do
  args=""
  IFS=';' read -ra KV <<< "$arm"
  for kv in "${KV[@]}"; do [ -n "$kv" ] && args="$args --kernel-opt $kv"; done
  rm -rf /tmp/kprof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof -o k --output-format csv \
      -- python3 "$ROOT/bench.py" --steps ${STEPS:-5} --warmup 2 $args > "$ROOT/gpurun_out/kprof_$i.log" 2>&1) \
      || { echo "PROF FAIL [$arm]"; tail -20 gpurun_out/kprof_$i.log; exit 4; }
  f=$(find /tmp/kprof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kstats_$i.csv
  python3 scripts/prof_summary.py gpurun_out/kstats_$i.csv $(( ${STEPS:-5} + 2 )) "arm [$arm]" > gpurun_out/kstats_$i.md
  echo "== arm $i [$arm]"; head -22 gpurun_out/kstats_$i.md | tail -16
  i=$((i+1))
done
