set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u scripts/diag/ab_kernel.py"
O=gpurun_out/ab1.json
: > $O
$A --kernel ring_wgrad --opt x3_wg_target=1536 >> $O 2>>gpurun_out/ab1.err || exit 1
$A --kernel ring_fwd --opt x3_c1_pipe=0,x3_c1_f16b=0 --opt x3_c1_pipe=1,x3_c1_f16b=0 --opt x3_c1_pipe=0,x3_c1_f16b=1 >> $O 2>>gpurun_out/ab1.err || exit 1
$A --kernel layer_bwd --layer 1 --opt x3_dg_target=2048 --opt x3_dg_target=4096 --opt x3_dg_target=1024 >> $O 2>>gpurun_out/ab1.err || exit 1
$A --kernel layer_bwd --layer 2 --opt x3_dg_target=2048 --opt x3_dg_target=4096 --opt x3_wg3_tile=0,x3_dg_target=2048 >> $O 2>>gpurun_out/ab1.err || exit 1
$A --kernel layer_bwd --layer 3 --opt x3_fc_dg_gemm=1 --opt x3_fc_dg_gemm=0 >> $O 2>>gpurun_out/ab1.err || exit 1
