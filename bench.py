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


SOLVE_KEYS = ("preset", "paths_per_gpu", "envs_per_path", "t_max", "N", "B", "trunk_scale", "env_reduction", "lr",
              "entropy_beta", "gae_lambda", "fitness", "concurrent_tournaments", "dtype", "rmsp_epsilon")


def solve_key(cfg, preset_name: str) -> dict:
    """The fields of a scripts/solve.py record that must equal the bench config for its
    generations-to-solve to be reported next to the bench's frames/s."""
    return {"preset": preset_name, "paths_per_gpu": cfg.paths, "envs_per_path": cfg.envs_per_path,
            "t_max": cfg.a2c.t_max, "N": cfg.net.N, "B": cfg.ga.B, "trunk_scale": cfg.net.trunk_scale,
            "env_reduction": cfg.a2c.env_reduction, "lr": round(float(cfg.a2c.lr), 8),
            "entropy_beta": cfg.a2c.entropy_beta, "gae_lambda": cfg.a2c.gae_lambda, "fitness": cfg.ga.fitness,
            "concurrent_tournaments": cfg.ga.concurrent_tournaments, "dtype": cfg.compute_dtype,
            "rmsp_epsilon": cfg.a2c.rmsp_epsilon}


def solve_records(key: dict, n_gpus: int):
    """Every committed solve run (profiles/solve/*.json, written by scripts/solve.py --out) whose config equals
    ``key`` on ``n_gpus`` GPUs -- solved or not, every seed -- or None when no run of this exact config exists."""
    import glob
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "solve")
    runs = []
    for f in sorted(glob.glob(os.path.join(root, "*.json"))):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        c = d.get("config") or {}
        if d.get("metric") != "generations_to_solve" or d.get("n_gpus") != n_gpus or not c.get("ga", True) \
                or c.get("same_path"):
            continue
        c = dict(c, dtype=c.get("dtype", "bf16"), lr=round(float(c.get("lr", 0.0)), 8),
                 rmsp_epsilon=c.get("rmsp_epsilon", 0.1))
        if any(c.get(k) != key[k] for k in SOLVE_KEYS):
            continue
        runs.append({"seed": c.get("seed"), "solved": bool(d.get("solved")),
                     "generations": d.get("generations_to_solve"), "frames": d.get("frames_to_solve"),
                     "seconds": d.get("seconds_to_solve"), "best_winner": d.get("best_winner_fitness"),
                     "budget_s": d.get("seconds"), "file": os.path.relpath(f, os.path.dirname(root))})
    if not runs:
        return {"value": None, "note": "no scripts/solve.py run of exactly this config is committed", "config": key}
    gens = sorted(r["generations"] for r in runs if r["solved"])
    med = gens[len(gens) // 2] if gens and len(gens) * 2 > len(runs) else None
    return {"value": med, "statistic": "median over seeds (null unless most seeds solved)",
            "solved_seeds": len(gens), "seeds": len(runs), "runs": runs, "config": key}


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
    ap.add_argument("--env", default=None, help="train this task of the preset's suite instead of its first task")
    ap.add_argument("--kernel-opt", action="append", default=[],
                    help="kernel switch NAME=VALUE (fast_conv_set_*), for A/B measurements")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp32x"],
                    help="HIP engine compute dtype (fp32: the reference's precision, csrc/trunk_f32.hip)")
    ap.add_argument("--deterministic", action="store_true", help="fixed-order gradient reductions (bit-reproducible)")
    ap.add_argument("--rollout-groups", type=int, default=0,
                    help="path groups stepped on their own streams in the rollout (0 = auto, 1 = one stream)")
    ap.add_argument("--ga-backend", default="device", choices=["device", "host"],
                    help="device: GA kernels inside the update graph + pipelined host bookkeeping")
    ap.add_argument("--concurrent", type=int, default=None,
                    help="concurrent tournaments (default paths/16 -- per rank count, NOT scaled by the world size, so "
                         "the GA takes the same number of tournaments per update on 1, 2, 4 and 8 GPUs)")
    ap.add_argument("--prof-window", action="store_true",
                    help="launch marker kernels around the timed updates (scripts/prof_window.py summarises the "
                         "rocprofv3 kernel trace between them)")
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
    if args.env:
        cfg.env = args.env
        cfg.tasks = [args.env] + [t for t in cfg.tasks if t != args.env]
    cfg.paths = args.paths
    cfg.envs_per_path = args.envs
    cfg.a2c.t_max = args.tmax
    cfg.backend = args.backend
    cfg.use_graph = not args.no_graph
    cfg.frame_ring = args.ring
    cfg.ga.concurrent_tournaments = args.concurrent or max(1, cfg.paths // 16)
    cfg.ga.backend = args.ga_backend
    cfg.compute_dtype = args.dtype
    cfg.deterministic = args.deterministic
    cfg.rollout_groups = args.rollout_groups
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        ctx.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        tr.update()
    tr.flush()
    sync()
    gen0 = tr.pop.generation
    step0 = tr.global_step
    if args.prof_window:
        from pathnet_gym_amd.ops import _lib as _plib
        _plib.call("launch_prof_marker", 1, _plib.stream())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.update()
    tr.flush()                               # drain the pipelined host bookkeeping of the last update
    if args.prof_window:
        _plib.call("launch_prof_marker", 2, _plib.stream())
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
            "dtype": tr.compute_dtype,
            "data": (f"synthetic: on-device Atari-style {cfg.tasks[0]} simulator (210x160 RGB -> gray 160x120 x4 "
                     "stack), random-init weights") if len(cfg.net.input_shape) == 3 else
                    f"synthetic: on-device {cfg.tasks[0]}, random-init weights",
            "config": {
                "model": f"PathNet {cfg.net.L} layers ("
                         + " + ".join(f"{sp.kind} {sp.out}" + (f" {sp.kernel}x{sp.kernel}/{sp.stride}"
                                                                 if sp.kind == "conv" else "")
                                      for sp in cfg.net.layers)
                         + f") x M={cfg.net.M} modules, N={cfg.net.N}, A2C T={cfg.a2c.t_max}, B={cfg.ga.B} tournament",
                "global_batch": B * ctx.world * cfg.a2c.t_max,
                "seq_len": cfg.a2c.t_max,
                "parallelism": f"dp{ctx.world} (population split: {cfg.paths} paths x {cfg.envs_per_path} envs per GPU)",
                "backend": args.backend,
                "hipgraph": cfg.use_graph,
                "frame_ring": bool(getattr(tr.engine, "ring", False)),
                "rollout_groups": int(getattr(tr.engine, "groups", 1)),
                "ga": f"{cfg.ga.backend} (B={cfg.ga.B}, {cfg.ga.concurrent_tournaments} concurrent tournaments)",
                "pipelined": bool(tr.pipelined),
                "deterministic": bool(getattr(tr.model.hip, "deterministic", False)),
            },
            "generations_in_timed_window": int(tr.pop.generation - gen0),
            # the metric's second half is measured by scripts/solve.py (minutes of training, not a bench window)
            "generations_to_solve": solve_records(solve_key(cfg, args.preset), ctx.world),
        }
        print(json.dumps(rec), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
