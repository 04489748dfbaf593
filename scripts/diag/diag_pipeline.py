#!/usr/bin/env python3
"""Locate implausible episode counters in the pipelined device-GA mode.

Every update: run the trainer's pipelined update, synchronise, then compare
(a) the device counters with a host recomputation from eng.dones / eng.epret,
(b) the host copy the pipeline collected one update later, and
(c) the fitness vectors, and report the first updates where any of them is
implausible (|return| > 21 for Pong).
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    from pathnet_gym_amd import _build
    _build.build()
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60
    graph = (sys.argv[2] != "nograph") if len(sys.argv) > 2 else True
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 16, 16, 5
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 1
    cfg.use_graph = graph
    tr = PathNetTrainer(cfg, device="cuda")
    eng = tr.engine
    t0 = time.time()
    n = 0
    reports = 0
    orig_collect = tr.comm.collect
    last = {}

    def collect(handle):
        fit, csum, stats = orig_collect(handle)
        last["csum"] = csum.copy()
        last["fit"] = fit.copy()
        return fit, csum, stats
    tr.comm.collect = collect
    prev_dev = None
    while time.time() - t0 < seconds:
        tr.update()
        torch.cuda.synchronize()
        d = eng.dones.bool()
        er = eng.epret[d]
        c_ref, s_ref = float(d.sum()), float(er.sum())
        c, s = float(eng.counters[1]), float(eng.counters[2])
        fit = eng.fitness.cpu().numpy()
        weird_fit = fit[(fit != -1000.0) & (np.abs(fit) > 21)]
        bad_dev = abs(c - c_ref) > 0.5 or abs(s - s_ref) > 1e-3 * max(1.0, abs(s_ref)) or abs(s) > 21 * max(c, 1)
        col = last.get("csum")
        # the collected counters belong to the previous update: compare with that update's device counters
        bad_col = col is not None and prev_dev is not None and (abs(col[1] - prev_dev[0]) > 0.5 or
                                                                abs(col[2] - prev_dev[1]) > 1e-3 * max(1.0, abs(prev_dev[1])))
        if (bad_dev or bad_col or len(weird_fit)) and reports < 12:
            reports += 1
            rec = {"update": n, "dev_counters": [c, s], "ref": [c_ref, s_ref], "collected": None if col is None else
                   [float(x) for x in col], "prev_dev": prev_dev, "weird_fit": weird_fit[:4].tolist(),
                   "max_abs_epret_done": float(er.abs().max()) if er.numel() else 0.0,
                   "epret_nonzero_not_done": int(((eng.epret != 0) & ~d).sum())}
            print(json.dumps(rec), flush=True)
        prev_dev = [c, s]
        n += 1
        if n % 500 == 0:
            print(json.dumps({"update": n, "t": round(time.time() - t0, 1), "reports": reports}), flush=True)
    print(json.dumps({"updates": n, "reports": reports}), flush=True)


if __name__ == "__main__":
    main()
