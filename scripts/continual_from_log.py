#!/usr/bin/env python3
"""Rebuild a scripts/continual.py result JSON from the run's stdout log.

Used for runs stopped at a job time limit before the JSON was written (continual.py now writes its JSON
after every phase).  Every number comes from the log lines the run printed: the per-task summary lines,
the per-task evaluation lines and the progress ("run") lines, which become the curves.

    python scripts/continual_from_log.py run.log out.json --config '{"paths": 16, ...}'
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("out")
    ap.add_argument("--config", default="{}", help="JSON object: the run's configuration (from its command line)")
    ap.add_argument("--note", default="")
    args = ap.parse_args()
    per_task, evals, curves, scratch = [], {}, {}, []
    for line in open(args.log):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "run" in d:
            if d["run"] == "sequence":
                curves.setdefault(d["task"], []).append(d)
            else:
                scratch.append(d)
        elif "updates" in d and "frozen_path" in d:
            per_task.append(d)
        elif "greedy_after_sequence" in d:
            evals[d["task"]] = d
        elif "updates" in d:                      # a finished scratch control
            scratch_done = d
            scratch_done["curve"] = scratch
            scratch = [scratch_done]
    for rec in per_task:
        rec["curve"] = curves.get(rec["task"], [])
        ev = evals.get(rec["task"], {})
        rec["greedy_after_sequence"] = ev.get("greedy_after_sequence")
        rec["frozen_params_bit_identical_at_end"] = ev.get("frozen_params_bit_identical_at_end")
        a, b = rec.get("greedy_after_task"), rec["greedy_after_sequence"]
        rec["forgetting"] = None if a is None or b is None else a - b
    controls = []
    if scratch and "updates" in scratch[0]:
        controls = scratch
    elif scratch:                                 # control stopped by the time limit: keep its curve, flagged
        last = scratch[-1]
        controls = [{"task": last["task"], "truncated": True, "frames": last["frames"],
                     "best_winner": last["best_winner"], "final_mean_return": last["mean_return"],
                     "solved": None, "curve": scratch}]
    out = {"experiment": "continual", "reference": "doom_pathnet.py:274-293, aliencentipede.txt:55-93",
           "stage": "rebuilt from log", "note": args.note, "tasks": [r["task"] for r in per_task],
           "n_gpus": 1, "config": json.loads(args.config), "per_task": per_task, "scratch_control": controls}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"tasks": out["tasks"], "controls": len(controls), "out": args.out}))


if __name__ == "__main__":
    main()
