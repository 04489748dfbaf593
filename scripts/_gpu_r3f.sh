set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
$T 300 $PYT tests/test_x3_engine.py > gpurun_out/r3/x3_tests_mm2.log 2>&1
tail -1 gpurun_out/r3/x3_tests_mm2.log
grep -q "failed" gpurun_out/r3/x3_tests_mm2.log && exit 1
PATHNET_X3_FC_MM=1 DT=fp32x TAG=x3_v8_mm bash scripts/gpu_r3_prof.sh > /dev/null
for t in x3_v8_mm; do sed -n 3p gpurun_out/r3/kwin_$t.md; grep "fc_fwd\|fc_slot" gpurun_out/r3/kwin_$t.md; done
bash scripts/_gpu_pmc_x3.sh > /dev/null 2>&1; tail -30 gpurun_out/r3/pmc_x3_summary.md; cat gpurun_out/r3/pmc_x3_mem.md | head -20
