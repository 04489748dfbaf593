set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "fused_fc_heads or gradient" tests/test_hip_kernels.py -k "heads or fused_fc_heads or gradient" > gpurun_out/t_heads2.log 2>&1 || { tail -30 gpurun_out/t_heads2.log; exit 1; }
tail -2 gpurun_out/t_heads2.log
bash scripts/diag/kwin.sh p8_h2 8 && bash scripts/diag/kwin.sh p64_h2 64
