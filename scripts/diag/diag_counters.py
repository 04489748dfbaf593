#!/usr/bin/env python3
"""Check the engine's episode counters against the stored rollout every update.

Recomputes (episodes, sum of finished-episode returns) from ``eng.dones`` /
``eng.epret`` on the host side of the same update and reports the first
mismatch or any implausible episode return, with the env's state row.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from pathnet_gym_amd import _build
    _build.build()
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 90
    cfg = preset("pong")
    cfg.ga.concurrent_tournaments = 4
    tr = PathNetTrainer(cfg, device="cuda")
    eng = tr.engine
    t0 = time.time()
    n = bad = 0
    while time.time() - t0 < seconds:
        eng.rollout_backward()
        torch.cuda.synchronize()
        d = eng.dones.bool()
        er = eng.epret[d]
        c_ref, s_ref = float(d.sum()), float(er.sum())
        c, s = float(eng.counters[1]), float(eng.counters[2])
        weird = er.abs().max().item() if er.numel() else 0.0
        if abs(c - c_ref) > 0.5 or abs(s - s_ref) > 1e-3 * max(1.0, abs(s_ref)) or weird > 21:
            bad += 1
            if bad <= 5:
                idx = torch.nonzero(d & (eng.epret.abs() > 21))[:3].tolist()
                st = eng.env._st32 if hasattr(eng.env, "_st32") else None
                print(json.dumps({"update": n, "counters": [c, s], "ref": [c_ref, s_ref], "max_abs_epret": weird,
                                  "bad_idx": idx,
                                  "state_rows": [st[i[1]].tolist() for i in idx] if st is not None else None}),
                      flush=True)
        fit_all, csum = tr.comm.exchange(eng.grad_flat, eng.fitness, eng.counters)
        if abs(float(csum[2]) - s) > 1e-3 * max(1.0, abs(s)):
            print(json.dumps({"update": n, "exchange_mismatch": [float(csum[2]), s]}), flush=True)
        eng.optimizer_step(cfg.a2c.lr)
        tr.global_step += int(csum[0])
        tr.updates += 1
        events = tr.pop.step(fit_all, tr.global_step)
        if events:
            tr._push_genotypes()
            lo, hi = tr.path_offset, tr.path_offset + tr.P
            eng.reset_fitness(torch.from_numpy(tr.pop.fitness[lo:hi]).to(tr.device))
        n += 1
        if n % 500 == 0:
            print(json.dumps({"update": n, "bad": bad, "t": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"updates": n, "bad_updates": bad}), flush=True)


if __name__ == "__main__":
    main()
