set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py tests/test_split_rollout.py tests/test_hip_kernels.py -k "x3 or heads or ring" > gpurun_out/t_lat.log 2>&1 || { tail -30 gpurun_out/t_lat.log; exit 1; }
tail -2 gpurun_out/t_lat.log
bash scripts/diag/kwin.sh p8_lat 8 && bash scripts/diag/kwin.sh p64_lat 64
