set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u scripts/diag/ab_kernel.py"
O=gpurun_out/ab_grids2.json
: > $O
for p in 8 64; do
  $A --paths $p --kernel layer_bwd --layer 2 --opt x3_wg3_target=512 --opt x3_wg3_target=256 --opt x3_wg3_target=1024 >> $O 2>>gpurun_out/ab_grids2.err || exit 1
  $A --paths $p --kernel layer_bwd --layer 4 --opt x3_fcw_target=2048 --opt x3_fcw_target=512 --opt x3_fcw_target=1024 >> $O 2>>gpurun_out/ab_grids2.err || exit 1
  $A --paths $p --kernel layer_bwd --layer 3 --opt py.fc_wgrad_gm_wgs=768 --opt py.fc_wgrad_gm_wgs=256 --opt py.fc_wgrad_gm_wgs=512 --opt py.fc_wgrad_gm_wgs=1536 >> $O 2>>gpurun_out/ab_grids2.err || exit 1
done
