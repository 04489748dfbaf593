# full validation on one MI355X: GPU tests, smoke, default bench, forced-RCCL vs no-group windows at 64 and 8 paths
set -o pipefail
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
for p in 64 8; do
  timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --windows 5 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build > $O/b_nogroup_p$p.json 2> $O/b_nogroup_p$p.err || exit 1
  PATHNET_DIST_FORCE=1 timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --windows 5 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build > $O/b_forced_p$p.json 2> $O/b_forced_p$p.err || exit 1
done
