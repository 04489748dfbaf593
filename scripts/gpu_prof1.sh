#!/bin/bash
# rocprofv3 kernel stats of one bench configuration.  Usage: ARGS="--no-ring" TAG=x scripts/gpu_prof1.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-p}
rm -rf /tmp/kprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof -o k --output-format csv \
    -- python3 "$ROOT/bench.py" --steps ${STEPS:-5} --warmup 2 ${ARGS:-} > "$ROOT/gpurun_out/kprof_$TAG.log" 2>&1) \
    || { echo "PROF FAIL"; tail -20 gpurun_out/kprof_$TAG.log; exit 4; }
f=$(find /tmp/kprof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kstats_$TAG.csv
t=$(find /tmp/kprof -name "*kernel_trace.csv" | head -1)
gzip -c "$t" > gpurun_out/ktrace_$TAG.csv.gz
python3 scripts/prof_summary.py gpurun_out/kstats_$TAG.csv $(( ${STEPS:-5} + 2 )) "$TAG [${ARGS:-}]" > gpurun_out/kstats_$TAG.md
head -20 gpurun_out/kstats_$TAG.md
tail -1 gpurun_out/kprof_$TAG.log
