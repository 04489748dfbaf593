# end-of-round validation: GPU suite, smoke, the driver's bench command, kernel windows at 64 / 8 paths, forced
# one-rank RCCL vs no group (medians of 5 windows, interleaved), the task-2 exchange on the forced group
set -o pipefail
OUT=gpurun_out/r6_final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest_gpu.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
OUT=$OUT bash scripts/gpu.sh "smoke" || exit 1
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log > $OUT/bench_default.json
python3 - $OUT/bench_default.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.get("strong_scaling") or {}
pr = (s.get("per_rank") or {}).get("by_n_gpus", {})
print("bench", d["value"], d["ms_per_step"], d["windows_ms_per_step"], "bf16", d.get("ms_per_step_bf16"),
      "ref", (d.get("reference_preset") or {}).get("ms_per_update"),
      "per_rank", {k: v["ms_per_update"] for k, v in pr.items()},
      "solve", {k: (d.get("generations_to_solve_in_run") or {}).get(k) for k in ("stopped", "generations_to_solve", "updates_to_solve", "heldout_mean")},
      "g2s", {k: (d.get("generations_to_solve") or {}).get(k) for k in ("value", "min", "max", "solved_seeds", "seeds")})
PY
for arm in nogroup forced nogroup forced; do
  for p in 8 64; do
    if [ $arm = forced ]; then export PATHNET_DIST_FORCE=1; else unset PATHNET_DIST_FORCE; fi
    timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --steps 20 --warmup 5 --windows 5 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build --no-strong > $OUT/rccl_${arm}_p$p.log 2>&1 || { echo "rccl bench $arm $p failed"; tail -20 $OUT/rccl_${arm}_p$p.log; exit 1; }
    grep '^{' $OUT/rccl_${arm}_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm p$p', d['ms_per_step'], d['windows_ms_per_step'])"
  done
done
unset PATHNET_DIST_FORCE
PATHNET_DIST_FORCE=1 timeout -k 10 300 python -u scripts/diag/task2_exchange.py --paths 8 > $OUT/task2_exchange_p8.log 2>&1 || { echo "task2 failed"; tail -20 $OUT/task2_exchange_p8.log; exit 1; }
tail -1 $OUT/task2_exchange_p8.log
KSTEPS=20 OUT=$OUT bash scripts/gpu.sh "kwin p64_final --per-rank-shapes '' --reference-preset 0 --no-verify-build" "kwin p8_final --paths 8 --paths-total 8 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
