# stall counters of one kernel via ab_kernel.py (two passes of <= 8 SQ counters):
#   pmc_kernel.sh LABEL MATCH ab_kernel-args...  -> gpurun_out/pmc_LABEL.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
L=$1; M=$2; shift 2
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
B="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS"
: > $R/gpurun_out/pmc_$L.txt
i=0
for C in "$A" "$B"; do
  i=$((i+1))
  rm -rf /tmp/pmck_$i
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/pmck_$i -o p -- python3 $R/scripts/diag/ab_kernel.py --rounds 1 --reps 3 "$@" > $R/gpurun_out/pmc_${L}_$i.log 2>&1 || exit 1
  f=$(find /tmp/pmck_$i -name "*counter_collection.csv" | head -1)
  python3 $R/scripts/pmc_dump.py $f --top 4 --match "$M" >> $R/gpurun_out/pmc_$L.txt || exit 1
done
