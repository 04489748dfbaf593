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

Precision: the headline runs the fp32x engine (``--dtype fp32x``, reported as
"dtype": "fp32"): the reference trains in fp32 (game_ac_network.py:89-110) and
fp32x matches a plain fp32 oracle to <= 2e-5 per layer (fp16 / bf16 hi+lo
operand pairs, three MFMAs per product, csrc/trunk_x3.hip).  The bf16 engine
is timed on the same config as ``value_bf16``.

Steady state: every env's first episode starts at a random late score
(PongVec.stagger_scores), so fitness windows fill and tournaments fire inside
the timed window (``generations_in_timed_window``).  After it, one
generations-to-solve seed runs on a fresh trainer under a hard wall cap
(``generations_to_solve_in_run``); ``generations_to_solve`` lists every
committed multi-seed record of exactly this config (scripts/solve.py).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
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


def build_trainer(args, ctx, dtype: str, stagger: bool):
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset(args.preset)
    if args.env:
        cfg.env = args.env
        cfg.tasks = [args.env] + [t for t in cfg.tasks if t != args.env]
    cfg.paths = args.paths
    cfg.envs_per_path = args.envs
    cfg.a2c.t_max = args.tmax
    cfg.backend = args.backend
    cfg.use_graph = not args.no_graph
    # fp32x: the first layer reads the frame ring (env 70 -> 39 us per step; conv1 forward / weight gradient +6 % /
    # +7 %; window 11.42 -> 11.15 ms, profiles/r3/kwin_x3_v19*.md); bf16 keeps packed stacks (a wash there, docs/PERF.md)
    cfg.frame_ring = args.ring or (dtype == "fp32x" and not args.packed)
    cfg.ga.concurrent_tournaments = args.concurrent or max(1, cfg.paths // 16)
    cfg.ga.backend = args.ga_backend
    cfg.compute_dtype = dtype
    cfg.deterministic = args.deterministic
    cfg.rollout_groups = args.rollout_groups
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
    if stagger and hasattr(tr.env, "stagger_scores"):
        tr.env.stagger_scores()
    return cfg, tr


def timed_window(tr, ctx, steps: int, warmup: int, markers: bool = False):
    """W untimed updates, then EXACTLY K updates between barrier + synchronize on both sides; max over ranks."""
    import torch

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        ctx.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for _ in range(warmup):
        tr.update()
    tr.flush()
    sync()
    gen0 = tr.pop.generation
    step0 = tr.global_step
    if markers:
        from pathnet_gym_amd.ops import _lib as _plib
        _plib.call("launch_prof_marker", 1, _plib.stream())
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.update()
    tr.flush()                               # drain the pipelined host bookkeeping of the last update
    if markers:
        _plib.call("launch_prof_marker", 2, _plib.stream())
    sync()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    return dt, tr.global_step - step0, tr.pop.generation - gen0   # whole-job agent steps (fused all-reduce)


def in_run_solve(args, ctx, dtype: str, cap_s: float) -> dict:
    """One seed of generations-to-solve on a FRESH trainer of the bench config, observed inside this run (hard wall
    cap; scripts/solve.py is the multi-seed version): the first tournament whose winner fitness reaches the task's
    reward threshold."""
    from pathnet_gym_amd.envs.registry import reward_threshold
    cfg, tr = build_trainer(args, ctx, dtype, stagger=False)
    thr = reward_threshold(cfg.tasks[0])
    t0 = time.time()
    last = t0
    best = -math.inf
    out = {"seed": cfg.seed, "threshold": thr, "cap_s": cap_s, "solved": False}
    while time.time() - t0 < cap_s:
        st = tr.update()
        now = time.time()
        if now - last > 30 and ctx.is_main:      # progress on stderr (the JSON line stays the only stdout line)
            last = now
            print(f"[bench] solve t={now - t0:.0f}s generation={tr.pop.generation} frames={tr.global_step} "
                  f"best_winner={best:.2f}", file=sys.stderr, flush=True)
        if st.tournaments:
            best = max(best, st.best_winner)
            if st.best_winner >= thr:
                out.update(solved=True, generations=tr.pop.generation, frames=tr.global_step,
                           seconds=round(time.time() - t0, 1))
                break
    tr.flush()
    out.update(best_winner=best if best > -math.inf else None, generations_run=tr.pop.generation,
               frames_run=tr.global_step, wall_s=round(time.time() - t0, 1))
    return out


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
    ap.add_argument("--packed", action="store_true", help="fp32x: packed 4-frame stacks instead of the frame ring")
    ap.add_argument("--preset", default="pong")
    ap.add_argument("--env", default=None, help="train this task of the preset's suite instead of its first task")
    ap.add_argument("--kernel-opt", action="append", default=[],
                    help="kernel switch NAME=VALUE (fast_conv_set_*), for A/B measurements")
    ap.add_argument("--dtype", default="fp32x", choices=["bf16", "fp32", "fp32x"],
                    help="HIP engine compute dtype.  fp32x (headline): fp32-accurate split operands (fp16 / bf16 "
                         "hi+lo pairs, 3 MFMAs per product, <= 2e-5 per layer vs a plain fp32 oracle, "
                         "csrc/trunk_x3.hip); fp32: fp32 MFMA operands (csrc/trunk_f32.hip); bf16: bf16 operands")
    ap.add_argument("--deterministic", action="store_true", help="fixed-order gradient reductions (bit-reproducible)")
    ap.add_argument("--rollout-groups", type=int, default=0,
                    help="path groups stepped on their own streams in the rollout (0 = auto, 1 = one stream)")
    ap.add_argument("--ga-backend", default="device", choices=["device", "host"],
                    help="device: GA kernels inside the update graph + pipelined host bookkeeping")
    ap.add_argument("--concurrent", type=int, default=None,
                    help="concurrent tournaments (default paths/16 -- per rank count, NOT scaled by the world size, so "
                         "the GA takes the same number of tournaments per update on 1, 2, 4 and 8 GPUs)")
    ap.add_argument("--no-stagger", action="store_true",
                    help="start every env at 0-0 (default: random late scores, so tournaments fire inside the window)")
    ap.add_argument("--solve-seconds", type=float, default=None,
                    help="after the timed window, run one generations-to-solve seed on a fresh trainer for at most "
                         "this long (default: up to 420 s on one GPU, within a 540 s total; 0 = off; multi-GPU "
                         "runs skip it)")
    ap.add_argument("--compare-bf16", type=int, default=None,
                    help="also time the bf16 engine on the same config (default: on for one GPU)")
    ap.add_argument("--prof-window", action="store_true",
                    help="launch marker kernels around the timed updates (scripts/prof_window.py summarises the "
                         "rocprofv3 kernel trace between them)")
    args = ap.parse_args()
    t_start = time.time()

    import torch

    from pathnet_gym_amd.parallel.dist import init_distributed

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
    single = ctx.world == 1 and not args.prof_window
    # the in-run solve may use what is left of a ~540 s budget (the driver allows 600 s for the whole bench; a fresh
    # box can spend a minute or two importing torch), at most 420 s
    solve_s = args.solve_seconds if args.solve_seconds is not None else (420.0 if single else 0.0)
    compare = args.compare_bf16 if args.compare_bf16 is not None else int(single and args.dtype != "bf16")
    stagger = not args.no_stagger
    cfg, tr = build_trainer(args, ctx, args.dtype, stagger)
    dt, frames, gens = timed_window(tr, ctx, args.steps, args.warmup, markers=args.prof_window)
    value = frames / dt
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
        "dtype": "fp32" if tr.compute_dtype == "fp32x" else tr.compute_dtype,
        "compute": {"fp32x": "fp32-accurate split operands: fp16 hi+lo pairs (forward), bf16 hi+lo pairs (gradients), "
                             "3 MFMAs per product, fp32 accumulation and master weights; <= 2e-5 relative per layer "
                             "vs a plain fp32 PyTorch oracle (tests/test_x3_engine.py)",
                    "fp32": "fp32 MFMA operands (v_mfma_f32_16x16x4_f32)",
                    "bf16": "bf16/fp16 MFMA operands, fp32 accumulation (reduced precision)"}[tr.compute_dtype],
        "data": (f"synthetic: on-device Atari-style {cfg.tasks[0]} simulator (210x160 RGB -> gray 160x120 x4 "
                 "stack), random-init weights") if len(cfg.net.input_shape) == 3 else
                f"synthetic: on-device {cfg.tasks[0]}, random-init weights",
        "config": {
            "model": f"PathNet {cfg.net.L} layers ("
                     + " + ".join(f"{sp.kind} {sp.out}" + (f" {sp.kernel}x{sp.kernel}/{sp.stride}"
                                                             if sp.kind == "conv" else "")
                                  for sp in cfg.net.layers)
                     + f") x M={cfg.net.M} modules, N={cfg.net.N}, A2C T={cfg.a2c.t_max}, B={cfg.ga.B} tournament",
            "global_batch": cfg.paths * cfg.envs_per_path * ctx.world * cfg.a2c.t_max,
            "seq_len": cfg.a2c.t_max,
            "parallelism": f"dp{ctx.world} (population split: {cfg.paths} paths x {cfg.envs_per_path} envs per GPU)",
            "backend": args.backend,
            "hipgraph": cfg.use_graph,
            "frame_ring": bool(getattr(tr.engine, "ring", False)),
            "rollout_groups": int(getattr(tr.engine, "groups", 1)),
            "ga": f"{cfg.ga.backend} (B={cfg.ga.B}, {cfg.ga.concurrent_tournaments} concurrent tournaments, "
                  f"fitness {cfg.ga.fitness} over {cfg.ga.window_for(cfg.envs_per_path)} episodes)",
            "pipelined": bool(tr.pipelined),
            "deterministic": bool(getattr(tr.model.hip, "deterministic", False)),
            "episode_stagger": stagger,
        },
        "generations_in_timed_window": int(gens),
    }
    del tr
    if compare:
        _, trb = build_trainer(args, ctx, "bf16", stagger)
        dtb, fb, _ = timed_window(trb, ctx, args.steps, args.warmup)
        rec["value_bf16"] = round(fb / dtb, 1)
        rec["ms_per_step_bf16"] = round(dtb / args.steps * 1e3, 3)
        del trb
    torch.cuda.empty_cache() if torch.cuda.is_available() else None
    # the metric's second half: one seed observed in this run, plus every committed multi-seed record of exactly
    # this config (scripts/solve.py --out profiles/solve/*.json)
    if solve_s > 0 and args.solve_seconds is None:
        solve_s = max(0.0, min(solve_s, 540.0 - (time.time() - t_start)))
    if solve_s > 0:
        rec["generations_to_solve_in_run"] = in_run_solve(args, ctx, args.dtype, solve_s)
    if ctx.is_main:
        rec["generations_to_solve"] = solve_records(solve_key(cfg, args.preset), ctx.world)
        print(json.dumps(rec), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
