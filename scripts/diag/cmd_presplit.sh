set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "gradient or dgrad" > gpurun_out/t_presplit.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/diag/ab_kernel.py --kernel layer_bwd --layer 1 --opt x3_presplit=0 --opt x3_presplit=1 > gpurun_out/ab_presplit.json 2> gpurun_out/ab_presplit.err || exit 1
timeout -k 10 300 python -u scripts/diag/ab_kernel.py --kernel layer_bwd --layer 2 --opt x3_presplit=0 --opt x3_presplit=1 >> gpurun_out/ab_presplit.json 2>> gpurun_out/ab_presplit.err
