set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
$T 300 $PYT tests/test_x3_engine.py > gpurun_out/r3/x3_tests_mm.log 2>&1
tail -1 gpurun_out/r3/x3_tests_mm.log
grep -q " passed" gpurun_out/r3/x3_tests_mm.log || exit 1
DT=fp32x TAG=x3_v6 bash scripts/gpu_r3_prof.sh > /dev/null && \
PATHNET_X3_FC_MM=0 DT=fp32x TAG=x3_v6_nomm bash scripts/gpu_r3_prof.sh > /dev/null
for t in x3_v6 x3_v6_nomm; do sed -n 3p gpurun_out/r3/kwin_$t.md; grep "fc_fwd\|fc_slot" gpurun_out/r3/kwin_$t.md; done
