set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "ring or band or swapped" > gpurun_out/t_fcs.log 2>&1 || exit 1
bash scripts/diag/kwin.sh p64_fcs 64 && bash scripts/diag/kwin.sh p8_fcs 8
