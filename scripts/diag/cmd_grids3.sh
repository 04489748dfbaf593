set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u scripts/diag/ab_kernel.py --reps 20"
O=gpurun_out/ab_grids3.json
: > $O
for p in 8 16 64; do
  $A --paths $p --kernel ring_fwd --opt x3_c1f_target=512,x3_c1f_minb=2 --opt x3_c1f_target=256,x3_c1f_minb=1 --opt x3_c1f_target=512,x3_c1f_minb=1 --opt x3_c1f_target=768,x3_c1f_minb=1 >> $O 2>>gpurun_out/ab_grids3.err || exit 1
  $A --paths $p --kernel conv23_fwd --opt x3_c23_target=512,x3_c23_mins=2 --opt x3_c23_target=512,x3_c23_mins=1 --opt x3_c23_target=256,x3_c23_mins=1 --opt x3_c23_target=1024,x3_c23_mins=1 >> $O 2>>gpurun_out/ab_grids3.err || exit 1
done
