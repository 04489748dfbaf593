# the driver's one-GPU bench command, as the driver runs it
set -o pipefail
OUT=gpurun_out/r6_final
mkdir -p $OUT
timeout -k 10 800 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default2.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_default2.log; exit 1; }
grep '^{' $OUT/bench_default2.log > $OUT/bench_default2.json
python3 - $OUT/bench_default2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("generations_to_solve_in_run") or {}
print("bench", d["value"], d["ms_per_step"], d["windows_ms_per_step"], "bf16", d.get("ms_per_step_bf16"),
      "ref", (d.get("reference_preset") or {}).get("ms_per_update"))
print("in-run solve", {k: r.get(k) for k in ("deterministic", "stopped", "generations_to_solve", "updates_to_solve", "heldout_mean", "wall_s")}, r.get("vs_committed"))
PY
