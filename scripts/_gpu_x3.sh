set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_x3_engine.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r3/x3_tests.log 2>&1
DT=fp32x TAG=x3_v2 bash scripts/gpu_r3_prof.sh && timeout -k 10 560 python bench.py > gpurun_out/r3/bench_full_v1.log 2>&1
