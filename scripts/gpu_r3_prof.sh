#!/bin/bash
# Steady-state rocprofv3 kernel trace of bench.py (timed window only).  Usage: DT=fp32x TAG=x3_v1 scripts/gpu_r3_prof.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
rm -rf /tmp/kprof
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/kprof -o k --output-format csv \
    -- python3 "$ROOT/bench.py" --steps ${STEPS:-10} --warmup 3 --dtype ${DT:-fp32x} --prof-window ${EXTRA:-} \
    > "$ROOT/gpurun_out/r3/prof_${TAG}.log" 2>&1) || { echo "PROF FAIL"; tail -20 gpurun_out/r3/prof_${TAG}.log; exit 4; }
f=$(find /tmp/kprof -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_window.py "$f" ${STEPS:-10} "${DT:-fp32x} bench, steady-state window ($TAG)" > gpurun_out/r3/kwin_${TAG}.md
head -30 gpurun_out/r3/kwin_${TAG}.md
