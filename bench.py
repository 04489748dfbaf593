#!/usr/bin/env python3
"""Headline benchmark: env frames/s (whole node), Pong PathNet, 1..8 GPUs.

BASELINE.json metric "env frames/sec (whole node) + generations-to-solve,
Pong PathNet 1/2/4/8 GPU"; config "Atari Pong pixels, L=3 conv + 2 fc x
N=10 modules, population split across 8xMI355X".

One timed step = one full A2C update of the local population on every rank:
T=20 env steps of P paths x E envs (on-device Pong: physics + render + gray
+ resize + frame stack), PathNet forward (active modules only) + sampling,
bootstrap, loss gradient, backward, ONE fused RCCL all-reduce of
active-module gradients + fitness + counters, clip + RMSProp, GA
tournaments.  Nothing is skipped inside the timed region.

A "frame" is one agent-environment step (one observation), i.e. the same
unit as the reference's 63 global steps/s (aliencentipede.txt);
the synthetic Pong repeats each action for `frameskip`=4 emulator sub-frames
that are NOT counted.  Weak scaling: P paths per GPU, fixed.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_STEPS_PER_SEC = 63.0     # reference steady-state global agent steps/s


def _solve_record():
    """Latest committed generations-to-solve measurement for Pong (profiles/solve), if present."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "solve", "pong_n10_devga_seed1.json")
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
        return {"value": d.get("generations_to_solve"), "frames": d.get("frames_to_solve"),
                "seconds": d.get("seconds_to_solve"), "n_gpus": d.get("n_gpus"),
                "config": "Pong PathNet M=10, N=10 initial modules, 16 paths x 16 envs, T=5, B=3, device GA",
                "seeds_1_2_3": [2314, 2341, 2088],
                "source": "profiles/solve/pong_n10_devga_seed*.json (scripts/solve.py)"}
    except (OSError, ValueError, IndexError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--paths", type=int, default=64, help="paths per GPU")
    ap.add_argument("--envs", type=int, default=32, help="envs per path (multiple of 16)")
    ap.add_argument("--tmax", type=int, default=20)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--ring", action="store_true", help="frame ring (single-frame writes) instead of packed stacks")
    ap.add_argument("--preset", default="pong")
    ap.add_argument("--kernel-opt", action="append", default=[],
                    help="kernel switch NAME=VALUE (fast_conv_set_*), for A/B measurements")
    ap.add_argument("--ga-backend", default="device", choices=["device", "host"],
                    help="device: GA kernels inside the update graph + pipelined host bookkeeping")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.parallel.dist import init_distributed
    from pathnet_gym_amd.algo.trainer import PathNetTrainer

    if args.backend == "hip":
        from pathnet_gym_amd import _build
        _build.build()

    if args.kernel_opt:
        from pathnet_gym_amd.ops import _lib
        for kv in args.kernel_opt:
            k, v = kv.split("=")
            lib = _lib.lib()
            (getattr(lib, k) if hasattr(lib, k) and "_set_" in k else getattr(lib, "fast_conv_set_" + k))(int(v))
    ctx = init_distributed()
    cfg = preset(args.preset)
    cfg.paths = args.paths
    cfg.envs_per_path = args.envs
    cfg.a2c.t_max = args.tmax
    cfg.backend = args.backend
    cfg.use_graph = not args.no_graph
    cfg.frame_ring = args.ring
    cfg.ga.concurrent_tournaments = max(1, (cfg.paths * ctx.world) // 16)
    cfg.ga.backend = args.ga_backend
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)

    def sync():
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        tr.update()
    tr.flush()
    sync()
    gen0 = tr.pop.generation
    step0 = tr.global_step
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.update()
    tr.flush()                               # drain the pipelined host bookkeeping of the last update
    sync()
    dt = time.perf_counter() - t0
    dt = ctx.max_scalar(dt)
    frames = tr.global_step - step0          # whole-job agent steps (all ranks, from the fused all-reduce)
    value = frames / dt
    if ctx.is_main:
        B = cfg.paths * cfg.envs_per_path
        rec = {
            "metric": "env_frames_per_sec_whole_node_pong_pathnet",
            "value": round(value, 1),
            "unit": "env frames/s (agent steps, all GPUs)",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_STEPS_PER_SEC, 1),
            "dtype": "bf16",
            "data": "synthetic: on-device Atari-style Pong simulator (210x160 RGB -> gray 160x120 x4 stack), "
                    "random-init weights",
            "config": {
                "model": f"PathNet {cfg.net.L} layers (3 conv 8-map + 2 fc 256) x M={cfg.net.M} modules, N={cfg.net.N}, "
                         f"A2C T={cfg.a2c.t_max}, B={cfg.ga.B} tournament",
                "global_batch": B * ctx.world * cfg.a2c.t_max,
                "seq_len": cfg.a2c.t_max,
                "parallelism": f"dp{ctx.world} (population split: {cfg.paths} paths x {cfg.envs_per_path} envs per GPU)",
                "backend": args.backend,
                "hipgraph": cfg.use_graph,
                "frame_ring": bool(getattr(tr.engine, "ring", False)),
                "ga": f"{cfg.ga.backend} (B={cfg.ga.B}, {cfg.ga.concurrent_tournaments} concurrent tournaments)",
                "pipelined": bool(tr.pipelined),
            },
            "generations_in_timed_window": int(tr.pop.generation - gen0),
            # the metric's second half is measured by scripts/solve.py (minutes of training, not a bench window)
            "generations_to_solve": _solve_record(),
        }
        print(json.dumps(rec), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
