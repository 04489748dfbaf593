set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
$T 300 $PYT tests/test_x3_engine.py > gpurun_out/r3/x3_tests_ks.log 2>&1
tail -1 gpurun_out/r3/x3_tests_ks.log
grep -q " passed" gpurun_out/r3/x3_tests_ks.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_ks.log && exit 1
DT=fp32x TAG=x3_v7 bash scripts/gpu_r3_prof.sh > /dev/null && \
DT=fp32x TAG=x3_v7_ks1 EXTRA="--kernel-opt fast_conv_set_x3_fc_ks=1" bash scripts/gpu_r3_prof.sh > /dev/null
for t in x3_v7 x3_v7_ks1; do sed -n 3p gpurun_out/r3/kwin_$t.md; grep "fc_fwd" gpurun_out/r3/kwin_$t.md; done
