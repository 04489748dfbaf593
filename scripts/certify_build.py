#!/usr/bin/env python3
"""Build-equivalence certificate for the committed generations-to-solve records.

The records of profiles/solve/ (scripts/solve.py, v2 criterion) carry the sources_sha256 of the build that ran them,
and bench.solve_records reports only records of the running build.  A kernel change that is bit-identical in the
deterministic fp32x mode (the mode every committed seed ran in) leaves every record valid, but changes the sha.  This
script proves such an equivalence the strong way: it re-runs one committed seed, deterministic, on the CURRENT build
(scripts/solve.py as a child process, the record's own config) and compares generations, updates, frames and the
held-out mean with the committed record of an older build.  Only an exact reproduction yields a certificate
``{"from": old_sha, "to": new_sha, "reproduces": true, ...}``; bench.solve_records then accepts the older build's
records for the newer build (profiles/solve/build_equivalence.json, entries appended by hand from the certificate).

    python scripts/certify_build.py --seed 1 --out-dir gpurun_out/cert
"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def committed(seed: int, root: str):
    """The newest deterministic v2 record of ``seed`` among the committed bench-config records."""
    best = None
    for f in sorted(glob.glob(os.path.join(root, "*.json"))):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        if not isinstance(d, dict):
            continue
        c = d.get("config") or {}
        if d.get("metric") != "generations_to_solve" or c.get("seed") != seed or not c.get("deterministic") \
                or not d.get("solved") or d.get("n_gpus") != 1:
            continue
        if best is None or d.get("finished_at", 0) > best[1].get("finished_at", 0):
            best = (f, d)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out-dir", default="gpurun_out/cert")
    ap.add_argument("--minutes", type=float, default=12.0)
    a = ap.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    sys.path.insert(0, ROOT)
    from pathnet_gym_amd import _build            # no torch / GPU in this process
    new_sha = _build.build_info(_build.build())["sources_sha256"]
    got = committed(a.seed, os.path.join(ROOT, "profiles", "solve"))
    if got is None:
        raise SystemExit(f"no committed deterministic record of seed {a.seed}")
    f, rec = got
    c = rec["config"]
    old_sha = (rec.get("build") or {}).get("sources_sha256")
    out = os.path.join(a.out_dir, f"seed{a.seed}_{new_sha}.json")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "scripts", "solve.py"), "--preset", c["preset"],
           "--paths", str(c["paths_per_gpu"]), "--envs", str(c["envs_per_path"]), "--ring", "--dtype", c["dtype"],
           "--ga-backend", "device", "--deterministic", "--seed", str(a.seed), "--minutes", str(a.minutes),
           "--report-every", "60", "--curve", out + "l", "--out", out]
    print("[certify]", " ".join(cmd), flush=True)
    rc = subprocess.run(cmd).returncode
    if rc != 0:
        raise SystemExit(f"solve.py exited {rc}")
    new = json.loads(open(out).read().strip().splitlines()[-1])
    keys = ("generations_to_solve", "updates_to_solve", "frames_to_solve", "heldout_mean")
    same = all(new.get(k) == rec.get(k) for k in keys) and new.get("solved")
    cert = {"from": old_sha, "to": (new.get("build") or {}).get("sources_sha256", new_sha), "seed": a.seed,
            "reproduces": bool(same), "committed_file": os.path.relpath(f, ROOT),
            "committed": {k: rec.get(k) for k in keys}, "rerun": {k: new.get(k) for k in keys},
            "rerun_file": os.path.relpath(out, ROOT),
            "evidence": "deterministic fp32x re-run of a committed seed on the new build (scripts/certify_build.py)"}
    open(os.path.join(a.out_dir, "certificate.json"), "w").write(json.dumps(cert) + "\n")
    print(json.dumps(cert), flush=True)
    sys.exit(0 if same else 3)


if __name__ == "__main__":
    main()
