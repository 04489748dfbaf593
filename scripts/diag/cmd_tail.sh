set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tail_tests.log 2>&1 || { tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -2 gpurun_out/tail_tests.log
bash scripts/diag/kwin.sh p8_tail 8 || exit 1
