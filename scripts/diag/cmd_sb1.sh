set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "band_f16_staging" > gpurun_out/t_sb1.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/diag/ab_kernel.py --kernel ring_fwd --reps 20 --opt x3_c1_sb1=0 --opt x3_c1_sb1=1 > gpurun_out/ab_sb1.json 2> gpurun_out/ab_sb1.err || exit 1
timeout -k 10 300 python -u scripts/diag/ab_kernel.py --paths 8 --kernel ring_fwd --reps 20 --opt x3_c1_sb1=0 --opt x3_c1_sb1=1 >> gpurun_out/ab_sb1.json 2>> gpurun_out/ab_sb1.err
