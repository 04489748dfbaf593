# stall counters of the 64-path update (graph off): two passes of <= 8 SQ counters -> gpurun_out/pmc_stalls_{a,b}.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P=${1:-64}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
B="SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS"
i=0
for C in "$A" "$B"; do
  i=$((i+1))
  rm -rf /tmp/pmc_$i
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/pmc_$i -o p -- python3 $R/bench.py --paths $P --paths-total $P --steps 2 --warmup 1 --windows 1 --no-graph --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build > $R/gpurun_out/pmc_stalls_$i.log 2>&1 || exit 1
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  python3 $R/scripts/pmc_dump.py $f --top 40 > $R/gpurun_out/pmc_stalls_p${P}_$i.txt || exit 1
done
