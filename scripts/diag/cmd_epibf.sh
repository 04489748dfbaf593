set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "band_f16_staging" > gpurun_out/t_epibf.log 2>&1 || { tail -30 gpurun_out/t_epibf.log; exit 1; }
tail -2 gpurun_out/t_epibf.log
: > gpurun_out/ab_epibf.json
for p in 64 8; do
timeout -k 10 300 python -u scripts/diag/ab_kernel.py --paths $p --kernel ring_fwd --reps 20 --rounds 8 --opt x3_c1_epibf=0 --opt x3_c1_epibf=2 >> gpurun_out/ab_epibf.json 2>> gpurun_out/ab_epibf.err || exit 1
done
