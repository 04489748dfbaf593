#!/bin/bash
# PMC passes over the bench (no graph, so counters attribute per dispatch); summary per kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {
  local tag=$1; shift
  rm -rf /tmp/bpmc_$tag
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc "$@" -d /tmp/bpmc_$tag -o pmc --output-format csv \
     -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-graph ${BENCH_ARGS:-} > "$ROOT/gpurun_out/bpmc_$tag.log" 2>&1) \
     || { echo "PMC $tag FAIL"; tail -5 gpurun_out/bpmc_$tag.log; return 1; }
  cp "$(find /tmp/bpmc_$tag -name '*counter_collection.csv' | head -1)" gpurun_out/bpmc_$tag.csv
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit 1
pass b SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum || exit 1
if [ -n "$MEM" ]; then
  pass c SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES FETCH_SIZE || exit 1
  pass d WRITE_SIZE SQ_WAVES || exit 1
  python3 scripts/pmc_summary.py --mem gpurun_out/bpmc_c.csv gpurun_out/bpmc_d.csv > gpurun_out/bpmc_mem.md
  cat gpurun_out/bpmc_mem.md
fi
python3 scripts/pmc_summary.py gpurun_out/bpmc_a.csv gpurun_out/bpmc_b.csv > gpurun_out/bpmc_summary.md
cat gpurun_out/bpmc_summary.md
