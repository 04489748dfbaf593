set -o pipefail
mkdir -p gpurun_out/r3
BENCH_ARGS="--dtype fp32x --solve-seconds 0 --compare-bf16 0" MEM=1 bash scripts/gpu_bench_pmc.sh > gpurun_out/r3/pmc_x3.txt 2>&1
rc=$?
cp gpurun_out/bpmc_summary.md gpurun_out/r3/pmc_x3_summary.md 2>/dev/null
cp gpurun_out/bpmc_mem.md gpurun_out/r3/pmc_x3_mem.md 2>/dev/null
cat gpurun_out/r3/pmc_x3.txt | head -60
exit $rc
