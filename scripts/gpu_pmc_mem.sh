#!/bin/bash
# Memory-path PMC passes over the bench (no graph): L2 read latency, TA/TCP stalls, VMEM queue depth.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {
  local tag=$1; shift
  rm -rf /tmp/mpmc_$tag
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc "$@" -d /tmp/mpmc_$tag -o pmc --output-format csv \
     -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-graph > "$ROOT/gpurun_out/mpmc_$tag.log" 2>&1) \
     || { echo "PMC $tag FAIL"; tail -5 gpurun_out/mpmc_$tag.log; return 1; }
  cp "$(find /tmp/mpmc_$tag -name '*counter_collection.csv' | head -1)" gpurun_out/mpmc_$tag.csv
}
pass e TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum \
       TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_WAVES SQ_WAVE_CYCLES || exit 1
pass f SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES || exit 1
python3 scripts/pmc_dump.py gpurun_out/mpmc_e.csv gpurun_out/mpmc_f.csv --top 8 > gpurun_out/mpmc_summary.md
cat gpurun_out/mpmc_summary.md
