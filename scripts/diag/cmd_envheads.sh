set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "folded_heads" > gpurun_out/t_envheads.log 2>&1 || { tail -40 gpurun_out/t_envheads.log; exit 1; }
tail -4 gpurun_out/t_envheads.log
for p in 8; do
  for f in 0 1; do
    PATHNET_FUSE_ENV_HEADS=$f timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --windows 5 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build > gpurun_out/b_eh${f}_p$p.json 2> gpurun_out/b_eh${f}_p$p.err || exit 1
  done
done
PATHNET_FUSE_ENV_HEADS=1 bash scripts/diag/kwin.sh p8_eh 8 && bash scripts/diag/kwin.sh p64_eh 64
