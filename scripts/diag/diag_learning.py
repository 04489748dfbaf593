#!/usr/bin/env python3
"""Learning diagnostic: same Pong config on the HIP engine and on the torch (autograd) backend.

Prints entropy / value loss / return / gradient norms per parameter group so a
learning failure can be attributed (env signal, loss, optimizer, wiring).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(backend, args):
    import torch
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset(args.preset)
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = args.paths, args.envs, args.tmax
    cfg.backend = backend
    cfg.use_graph = backend == "hip"
    cfg.ga.concurrent_tournaments = max(1, args.paths // 16)
    if args.lr:
        cfg.a2c.lr = args.lr
    if args.no_ga:
        cfg.ga.B = 10 ** 9     # never enough candidates -> no tournaments
    tr = PathNetTrainer(cfg, device="cuda")
    lay = tr.model.store.layout
    groups = {"heads": [s for s in lay.segments if s.layer < 0]}
    for l in range(cfg.net.L):
        groups[f"layer{l}"] = [s for s in lay.segments if s.layer == l]
    t0 = time.time()
    ema = None
    n = 0
    flat0 = tr.model.store.flat.detach().clone()
    while time.time() - t0 < args.seconds:
        if backend == "hip":
            eng = tr.engine
            st = tr.update()
            g = eng.grad_flat
        else:
            st = tr.update()
            g = tr.model.store.flat.grad if tr.model.store.flat.grad is not None else None
        n += 1
        if not math.isnan(st.mean_return):
            ema = st.mean_return if ema is None else 0.95 * ema + 0.05 * st.mean_return
        if n % args.every == 0:
            rec = dict(backend=backend, t=round(time.time() - t0, 1), updates=n, frames=tr.global_step,
                       entropy=round(st.entropy, 4), loss_v=round(st.loss_v, 4), loss_pi=round(st.loss_pi, 4),
                       ret=None if ema is None else round(ema, 3), gen=tr.pop.generation)
            if g is not None:
                for k, segs in groups.items():
                    rec["g_" + k] = round(float(sum(float(g[s.offset:s.offset + s.numel].norm()) ** 2
                                                    for s in segs)) ** 0.5, 5)
            d = tr.model.store.flat.detach() - flat0
            for k, segs in groups.items():
                rec["dw_" + k] = round(float(sum(float(d[s.offset:s.offset + s.numel].norm()) ** 2
                                                 for s in segs)) ** 0.5, 5)
            print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backends", default="hip,torch")
    ap.add_argument("--preset", default="pong")
    ap.add_argument("--paths", type=int, default=16)
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--tmax", type=int, default=20)
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--every", type=int, default=50)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--no-ga", action="store_true")
    args = ap.parse_args()
    from pathnet_gym_amd import _build
    _build.build()
    for b in args.backends.split(","):
        run(b, args)


if __name__ == "__main__":
    main()
