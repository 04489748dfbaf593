# rollout groups sweep at small populations (fp32x frame ring)
set -o pipefail
mkdir -p gpurun_out
for cfg in "8 4" "16 4" "32 2" "32 1" "8 2" "8 1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --paths $1 --paths-total $1 --steps 20 --warmup 5 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build --rollout-groups $2 > gpurun_out/b3_p$1_g$2.json 2> gpurun_out/b3_p$1_g$2.err || exit 1
done
