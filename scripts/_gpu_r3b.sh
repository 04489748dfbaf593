set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
$T 300 $PYT tests/test_pipeline_guard.py > gpurun_out/r3/guard_tests.log 2>&1
PATHNET_OVERLAP_TRACE=gpurun_out/r3/overlap_trace_2rank.json $T 400 $PYT tests/test_dist_hip.py > gpurun_out/r3/dist_tests.log 2>&1
SEL="oracle or forward or backward or lstm or conv_gradients"
for i in 1 2; do
  PATHNET_RECORD_NUMERICS=gpurun_out/r3/numerics_measured.json $T 400 $PYT tests/test_hip_kernels.py tests/test_f32_engine.py -k "$SEL" > gpurun_out/r3/numerics_rec$i.log 2>&1 || exit 1
done
DT=fp32x TAG=x3_v5 bash scripts/gpu_r3_prof.sh > /dev/null
