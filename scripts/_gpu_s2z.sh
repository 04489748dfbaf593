#!/bin/bash
# End-of-session check: full GPU suite, smoke, the driver-contract bench (no in-run solve), a rocprofv3 --stats
# profile of the bench and the steady-state kernel window.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 \
    || { tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log | cut -c1-160
$T 300 python -u bench.py --steps 20 --warmup 5 --solve-seconds 0 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err \
    || { tail -20 gpurun_out/final/bench.err; exit 1; }
cut -c1-400 gpurun_out/final/bench.json
ROOT=$(pwd)
(cd /tmp && $T 300 rocprofv3 --kernel-trace --stats -d /tmp/fprof -o f --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --solve-seconds 0 --compare-bf16 0 > "$ROOT/gpurun_out/final/prof_bench.log" 2>&1) \
    || { echo "PROF FAIL"; tail -5 gpurun_out/final/prof_bench.log; exit 1; }
f=$(find /tmp/fprof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/final/kernel_stats.csv
DT=fp32x TAG=x3_final bash scripts/gpu_r3_prof.sh > /dev/null && sed -n 3p gpurun_out/r3/kwin_x3_final.md | cut -c100-
