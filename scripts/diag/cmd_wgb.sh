set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "gradient" > gpurun_out/t_wgb.log 2>&1 || { tail -30 gpurun_out/t_wgb.log; exit 1; }
tail -2 gpurun_out/t_wgb.log
bash scripts/diag/kwin.sh p64_wgb 64 && bash scripts/diag/kwin.sh p8_wgb 8
