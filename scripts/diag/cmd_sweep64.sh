set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/sweep64.json
: > $O
timeout -k 10 200 python -u scripts/diag/ab_kernel.py --paths 64 --kernel ring_wgrad --reps 5 --opt x3_wgrad_pf=3 --opt x3_wgrad_pf=2 --opt x3_wgrad_pf=1 >> $O 2>> $O.err || exit 1
timeout -k 10 200 python -u scripts/diag/ab_kernel.py --paths 64 --kernel layer_bwd --layer 1 --reps 10 --opt x3_wgrad_pf=3 --opt x3_wgrad_pf=2 --opt x3_wgrad_pf=1 >> $O 2>> $O.err || exit 1
timeout -k 10 200 python -u scripts/diag/ab_kernel.py --paths 64 --kernel layer_fwd --layer 4 --reps 20 --opt x3_fc_d=4 --opt x3_fc_d=2 --opt x3_fc_d=8 >> $O 2>> $O.err || exit 1
timeout -k 10 200 python -u scripts/diag/ab_kernel.py --paths 64 --kernel ring_wgrad --reps 5 --opt x3_c1_wg_ncx=2 --opt x3_c1_wg_ncx=1 >> $O 2>> $O.err || exit 1
