# end-of-round validation, part 1: the GPU suite, smoke and the driver's bench command (part 2: cmd_r6_final2.sh)
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
