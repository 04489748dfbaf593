set -o pipefail
bash scripts/diag/cmd_ab_libs.sh x0 x1 ab_fcw_xcd_p64.json --paths 64 --kernel layer_bwd --layer 3 --part w --reps 10 || exit 1
bash scripts/diag/cmd_ab_libs.sh x0 x1 ab_fcw_xcd_p8.json --paths 8 --kernel layer_bwd --layer 3 --part w --reps 20 || exit 1
