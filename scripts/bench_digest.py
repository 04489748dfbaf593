"""One-screen digest of a bench.py JSON record (the driver's one-GPU command): headline, bf16, reference preset,
per-rank strong-scaling shapes, the in-run solve against its committed record, and generations-to-solve.

    python scripts/bench_digest.py gpurun_out/.../bench_driver.json
"""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    s = d.get("strong_scaling") or {}
    pr = (s.get("per_rank") or {}).get("by_n_gpus", {})
    r = d.get("generations_to_solve_in_run") or {}
    g = d.get("generations_to_solve") or {}
    print("bench", d["value"], d["ms_per_step"], d["windows_ms_per_step"], "bf16", d.get("ms_per_step_bf16"),
          "ref", (d.get("reference_preset") or {}).get("ms_per_update"),
          "per_rank", {k: v["ms_per_update"] for k, v in pr.items()})
    print("in-run solve", {k: r.get(k) for k in ("deterministic", "stopped", "generations_to_solve", "updates_to_solve",
                                                   "heldout_mean", "wall_s")}, r.get("vs_committed"))
    print("g2s", {k: g.get(k) for k in ("value", "min", "max", "solved_seeds", "seeds", "excluded")})


if __name__ == "__main__":
    main(sys.argv[1])
