set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "ring" > gpurun_out/t_wgauto.log 2>&1 || { tail -30 gpurun_out/t_wgauto.log; exit 1; }
tail -2 gpurun_out/t_wgauto.log
: > gpurun_out/ab_wgauto.json
for p in 8 16 32 64; do
  timeout -k 10 300 python -u scripts/diag/ab_kernel.py --paths $p --kernel ring_wgrad --opt x3_wg_auto=1,x3_wg_target=1536 --opt x3_wg_auto=0,x3_wg_target=1536 --opt x3_wg_auto=0,x3_wg_target=3072 >> gpurun_out/ab_wgauto.json 2>> gpurun_out/ab_wgauto.err || exit 1
done
