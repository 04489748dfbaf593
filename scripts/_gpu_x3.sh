set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_x3_engine.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r3/x3_tests.log 2>&1
DT=fp32x TAG=x3_v1 bash scripts/gpu_r3_prof.sh && DT=bf16 TAG=bf16_v0 bash scripts/gpu_r3_prof.sh
