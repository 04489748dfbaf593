set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_x3_engine.py -x -q --timeout 300 --timeout-method thread > gpurun_out/refresh_tests.log 2>&1 || { tail -30 gpurun_out/refresh_tests.log; exit 1; }
tail -2 gpurun_out/refresh_tests.log
bash scripts/diag/kwin.sh p8_refresh 8 || exit 1
