set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_x3_engine.py tests/test_pipeline_guard.py tests/test_hip_kernels.py::test_rmsprop_kernel_matches_torch -v -s --timeout 120 --timeout-method thread > gpurun_out/r3/x3_tests.log 2>&1
PATHNET_OVERLAP_TRACE=gpurun_out/r3/overlap_trace_2rank.json timeout -k 10 400 python -u -m pytest tests/test_dist_hip.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r3/dist_tests.log 2>&1
DT=fp32x TAG=x3_v4 bash scripts/gpu_r3_prof.sh > /dev/null && \
DT=fp32x TAG=x3_v4_fcd2 EXTRA="--kernel-opt fast_conv_set_x3_fc_d=2" bash scripts/gpu_r3_prof.sh > /dev/null && \
DT=fp32x TAG=x3_v4_pf1 EXTRA="--kernel-opt fast_conv_set_x3_wgrad_pf=1" bash scripts/gpu_r3_prof.sh > /dev/null
