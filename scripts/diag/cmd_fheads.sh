set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "fused_fc_heads" > gpurun_out/t_fheads.log 2>&1 || { tail -40 gpurun_out/t_fheads.log; exit 1; }
tail -4 gpurun_out/t_fheads.log
A="timeout -k 10 300 python -u scripts/diag/ab_kernel.py --reps 20"
: > gpurun_out/ab_fh.json
for p in 64 8; do
  $A --paths $p --kernel fc_then_heads >> gpurun_out/ab_fh.json 2>> gpurun_out/ab_fh.err || exit 1
  $A --paths $p --kernel fc_heads --opt x3_fh_d=2 --opt x3_fh_d=3 >> gpurun_out/ab_fh.json 2>> gpurun_out/ab_fh.err || exit 1
done
for p in 64 8; do
  for f in 0 1; do
    PATHNET_X3_FUSE_HEADS=$f timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --windows 5 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build > gpurun_out/b_fh${f}_p$p.json 2> gpurun_out/b_fh${f}_p$p.err || exit 1
  done
done
