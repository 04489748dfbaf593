set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "gradient or wgrad or ring" > gpurun_out/t_pmap.log 2>&1 || exit 1
bash scripts/diag/kwin.sh p64_pmap1 64 && bash scripts/diag/kwin.sh p64_pmap0 64 --kernel-opt x3_slab_pmap=0 && bash scripts/diag/kwin.sh p64_pmap1b 64
