set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "rccl or pipelin or bench or trainer or x3_range or checkpoint" -x -q --timeout 300 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 || { tail -30 gpurun_out/pack_tests.log; exit 1; }
tail -2 gpurun_out/pack_tests.log
bash scripts/diag/kwin.sh p8_pack 8 || exit 1
