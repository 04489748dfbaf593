#!/bin/bash
# End-of-session extras on a GPU box: per-kernel PMC summaries of the bench (no graph) and the fp32 /
# deterministic bf16 bench lines.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
MEM=1 bash scripts/gpu_bench_pmc.sh > gpurun_out/pmc_final.log 2>&1 || { echo "PMC FAIL"; tail -20 gpurun_out/pmc_final.log; exit 1; }
echo pmc ok
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/bench_fp32.log 2>&1 \
    || { echo "FP32 BENCH FAIL"; tail -20 gpurun_out/bench_fp32.log; exit 1; }
tail -1 gpurun_out/bench_fp32.log | cut -c1-200
timeout -k 10 300 python -u bench.py --deterministic --steps 10 --warmup 3 > gpurun_out/bench_det.log 2>&1 \
    || { echo "DET BENCH FAIL"; tail -20 gpurun_out/bench_det.log; exit 1; }
tail -1 gpurun_out/bench_det.log | cut -c1-200
