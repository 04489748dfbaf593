#!/usr/bin/env python3
"""Generations-to-solve: the second half of the BASELINE.json headline metric.

"Solved" (the reference defines no criterion; algo/solve.py): the first GA tournament whose
winner fitness reaches the env's ``reward_threshold`` (Pong 18, CartPole-v1 475; the registry spirit of
gym_doom/__init__.py:21-90) AND whose winning path, evaluated held-out on --confirm-episodes fresh episodes with the
same weights, reaches --confirm.  Training stops at the task horizon, where the lr anneal reaches 0 (the reference's
task end, doom_pathnet.py:197,230): a run still unconfirmed there is "unsolved at horizon".  Reported as tournaments
("generations"), updates, agent frames and wall seconds until solve, every held-out check, and a learning curve in
JSONL.

    python scripts/solve.py --preset pong --minutes 15 [--paths 64 --envs 32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/solve.py ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="pong")
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--paths", type=int, default=None, help="paths per GPU (weak scaling)")
    ap.add_argument("--paths-total", type=int, default=None,
                    help="strong scaling: this population split over the GPUs (TrainConfig.paths_total)")
    ap.add_argument("--checkpoint", default=None, help="save the trainer here at the end (and every --ckpt-minutes)")
    ap.add_argument("--ckpt-minutes", type=float, default=0.0)
    ap.add_argument("--resume", action="store_true",
                    help="continue from --checkpoint (continuation resume, not bit-exact: weights, optimizer, GA and RNG "
                         "counters restored; light checkpoints rebuild each env's frame stack from its current frame "
                         "and, at momentum 0, hold no momentum slots); the "
                         "record's seconds / segments accumulate over the resumed runs (read back from --out)")
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--tmax", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--B", type=int, default=None)
    ap.add_argument("--env-reduction", default=None, choices=["sum", "mean_env"])
    ap.add_argument("--entropy-beta", type=float, default=None)
    ap.add_argument("--trunk-scale", default=None, choices=["M", "none"])
    ap.add_argument("--gae-lambda", type=float, default=None)
    ap.add_argument("--rmsp-eps", type=float, default=None, help="RMSProp epsilon (reference 0.1, inside the sqrt)")
    ap.add_argument("--grad-scale", type=float, default=None,
                    help="factor on the loss weight; 1/8 with --paths 512 emulates 8 ranks whose all-reduced "
                         "gradient is averaged (--rank-reduction mean) on one GPU")
    ap.add_argument("--rank-reduction", default=None, choices=["sum", "mean"])
    ap.add_argument("--concurrent", type=int, default=None,
                    help="concurrent tournaments (default paths/16 per rank count, independent of the world size)")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--curve", default="gpurun_out/solve_curve.jsonl")
    ap.add_argument("--report-every", type=float, default=30.0, help="seconds between progress lines")
    ap.add_argument("--keep-going", action="store_true", help="continue after solving until --minutes")
    ap.add_argument("--debug", action="store_true", help="inspect engine buffers on counter anomalies")
    ap.add_argument("--no-ga", action="store_true", help="disable tournaments (pure A2C on fixed paths)")
    ap.add_argument("--N", type=int, default=None, help="active modules per layer in the initial genotypes")
    ap.add_argument("--fitness", default=None, choices=["last", "mean"])
    ap.add_argument("--ga-backend", default=None, choices=["host", "device"])
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--fitness-window", type=int, default=None)
    ap.add_argument("--same-path", action="store_true",
                    help="every path starts from the same random N-module genotype (ablation)")
    ap.add_argument("--out", default=None, help="also write the final JSON record to this file")
    ap.add_argument("--ring", action="store_true", help="first layer on the frame ring (the fp32x bench default)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32", "fp32x"], help="HIP engine compute dtype")
    ap.add_argument("--deterministic", action="store_true", help="fixed-order gradient reductions")
    ap.add_argument("--confirm", type=float, default=17.0,
                    help="held-out mean return that confirms a solve candidate (algo/solve.py)")
    ap.add_argument("--confirm-episodes", type=int, default=64, help="fresh episodes of the held-out confirmation")
    args = ap.parse_args()

    import torch
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.envs.registry import reward_threshold
    from pathnet_gym_amd.parallel.dist import init_distributed
    from pathnet_gym_amd.algo.trainer import PathNetTrainer

    ctx = init_distributed()
    cfg = preset(args.preset)
    for k, v in (("paths", args.paths), ("envs_per_path", args.envs)):
        if v is not None:
            setattr(cfg, k, v)
    if args.tmax is not None:
        cfg.a2c.t_max = args.tmax
    if args.lr is not None:
        cfg.a2c.lr = args.lr
    if args.B is not None:
        cfg.ga.B = args.B
    if args.env_reduction is not None:
        cfg.a2c.env_reduction = args.env_reduction
    if args.entropy_beta is not None:
        cfg.a2c.entropy_beta = args.entropy_beta
    if args.trunk_scale is not None:
        cfg.net.trunk_scale = args.trunk_scale
    if args.gae_lambda is not None:
        cfg.a2c.gae_lambda = args.gae_lambda
    if args.rmsp_eps is not None:
        cfg.a2c.rmsp_epsilon = args.rmsp_eps
    if args.grad_scale is not None:
        cfg.a2c.grad_scale = args.grad_scale
    if args.rank_reduction is not None:
        cfg.a2c.rank_reduction = args.rank_reduction
    if args.N is not None:
        cfg.net.N = args.N
    if args.fitness is not None:
        cfg.ga.fitness = args.fitness
    if args.ga_backend is not None:
        cfg.ga.backend = args.ga_backend
    if args.seed is not None:
        cfg.seed = args.seed
        cfg.ga.seed = args.seed
    if args.fitness_window is not None:
        cfg.ga.fitness_window = args.fitness_window
    cfg.backend = args.backend
    cfg.use_graph = not args.no_graph
    cfg.frame_ring = bool(args.ring)
    if args.dtype is not None:
        cfg.compute_dtype = args.dtype
    cfg.deterministic = bool(args.deterministic)
    if args.paths_total:
        cfg.paths_total = args.paths_total
    cfg.ga.concurrent_tournaments = args.concurrent or max(1, (cfg.paths_total or cfg.paths) // 16)
    build_info = None
    if cfg.backend in ("hip", "auto") and ctx.device.type == "cuda":
        from pathnet_gym_amd import _build
        build_info = _build.build_info(_build.build())
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
    if args.no_ga:
        tr.pop.step = lambda *a, **k: []
        if tr.engine is not None and tr.engine.ga_dev is not None:
            tr.pop.slots[:] = -1                 # no tournament slots: the device GA never fires
            tr.engine.ga_upload(tr.pop)
    if args.same_path:
        tr.pop.genotypes[:] = tr.pop.genotypes[0]
        tr._push_genotypes()
        if tr.engine is not None and tr.engine.ga_dev is not None:
            tr.engine.ga_upload(tr.pop)
    prior = {"seconds": 0.0, "segments": []}
    if args.resume and args.checkpoint and os.path.exists(args.checkpoint):
        from pathnet_gym_amd.utils import checkpoint as ckpt
        ckpt.load(tr, args.checkpoint)
        if args.out and os.path.exists(args.out):
            with open(args.out) as f:
                old = json.loads(f.read().strip().splitlines()[-1])
            prior = {"seconds": float(old.get("seconds", 0.0)), "segments": list(old.get("segments", []))
                     or [{"updates": old.get("updates"), "seconds": old.get("seconds")}],
                     "best": old.get("best_winner_fitness"), "ema": old.get("final_mean_return"),
                     "candidates": list(old.get("candidates", []))}
        if ctx.is_main:
            print(json.dumps({"resumed": args.checkpoint, "updates": tr.updates, "generation": tr.pop.generation,
                              "frames": tr.global_step, "prior_seconds": prior["seconds"]}), flush=True)
    thr = reward_threshold(cfg.tasks[0])
    curve = None
    if ctx.is_main and args.curve:
        os.makedirs(os.path.dirname(args.curve) or ".", exist_ok=True)
        curve = open(args.curve, "a" if args.resume else "w")

    from pathnet_gym_amd.algo.solve import SolveTracker
    t0 = time.time()
    last = t0
    last_ckpt = t0
    u0 = tr.updates

    def log_candidate(c):
        if ctx.is_main:
            print(json.dumps({"candidate": c}), flush=True)
            if curve:
                curve.write(json.dumps({"candidate": c}) + "\n")
                curve.flush()

    trk = SolveTracker(tr, confirm_threshold=args.confirm, confirm_episodes=args.confirm_episodes,
                       wall_s=args.minutes * 60 - prior["seconds"], log=log_candidate)
    if prior.get("best") is not None:
        trk.best = prior["best"]
    trk.candidates = list(prior.get("candidates", []))     # the held-out checks of earlier segments
    ret_ema = prior.get("ema")
    while True:
        st = tr.update()
        if not math.isnan(st.mean_return) and abs(st.mean_return) > 1000 and ctx.is_main:
            rec = {"anomaly": "mean_return", "value": st.mean_return, "episodes": st.episodes, "update": tr.updates}
            eng = tr.engine
            if eng is not None and args.debug:
                d = eng.dones.bool()
                er = eng.epret[d]
                rec.update(ref_count=int(d.sum()), ref_sum=float(er.sum()), counters=eng.counters.tolist(),
                           big=torch.nonzero(d & (eng.epret.abs() > 21))[:4].tolist(),
                           big_vals=eng.epret[d & (eng.epret.abs() > 21)][:4].tolist(),
                           nonzero_epret_not_done=int(((eng.epret != 0) & ~d).sum()))
            print(json.dumps(rec), flush=True)
        elif not math.isnan(st.mean_return):
            ret_ema = st.mean_return if ret_ema is None else 0.9 * ret_ema + 0.1 * st.mean_return
        stop = trk.observe(st)       # a confirmed solve, the task horizon or the wall limit (same on every rank)
        if stop and trk.stopped == "solved" and args.keep_going:
            stop = trk.frames_in_task() >= trk.horizon
        now = time.time()
        if now - last >= args.report_every or stop:
            last = now
            rec = dict(t=round(prior["seconds"] + now - t0, 1), frames=tr.global_step, updates=tr.updates,
                       generation=tr.pop.generation, mean_return=ret_ema,
                       best_winner=trk.best if math.isfinite(trk.best) else None,
                       lr=trk.lr_now(tr.global_step), entropy=st.entropy,
                       frames_per_sec=round((tr.global_step - trk.tr.task_start_step) / max(now - t0, 1e-9), 1))
            if ctx.is_main:
                print(json.dumps(rec), flush=True)
                if curve:
                    curve.write(json.dumps(rec) + "\n")
                    curve.flush()
        if stop:
            break                                # replicated decisions: every rank breaks at the same update
        if args.checkpoint and args.ckpt_minutes > 0 and tr.updates % 32 == 0 and \
                ctx.max_scalar(now - last_ckpt) > args.ckpt_minutes * 60:
            from pathnet_gym_amd.utils import checkpoint as ckpt
            tr.flush()
            ckpt.save(tr, args.checkpoint, light=True)
            last_ckpt = time.time()
    tr.flush()
    if args.checkpoint:
        # a continuation checkpoint (no frame stacks, no momentum slots at momentum 0: ~45 MB at the bench network, not
        # 1.3 GB at 512 x 32 envs); the resumed run restarts every env's stack from its current frame
        from pathnet_gym_amd.utils import checkpoint as ckpt
        ckpt.save(tr, args.checkpoint, light=True)
    el = prior["seconds"] + time.time() - t0
    if ctx.is_main:
        r = trk.record()
        out = {"metric": "generations_to_solve", "env": cfg.tasks[0], "finished_at": round(time.time(), 1)}
        out.update(r)
        out.update({"final_mean_return": ret_ema, "generations": tr.pop.generation,
                    "frames": tr.global_step, "updates": tr.updates,
                    "seconds": round(el, 1), "n_gpus": ctx.world,
                    "segments": prior["segments"] + [{"updates": tr.updates - u0, "seconds": round(time.time() - t0, 1)}],
                    "config": {"preset": args.preset, "paths_per_gpu": cfg.paths, "envs_per_path": cfg.envs_per_path,
                               "t_max": cfg.a2c.t_max, "lr": cfg.a2c.lr, "B": cfg.ga.B,
                               "concurrent_tournaments": cfg.ga.concurrent_tournaments, "backend": tr.backend,
                               "env_reduction": cfg.a2c.env_reduction, "entropy_beta": cfg.a2c.entropy_beta,
                               "trunk_scale": cfg.net.trunk_scale, "gae_lambda": cfg.a2c.gae_lambda,
                               "rmsp_epsilon": cfg.a2c.rmsp_epsilon, "grad_scale": cfg.a2c.grad_scale,
                               "rank_reduction": cfg.a2c.rank_reduction,
                               "frame_ring": bool(getattr(tr.engine, "ring", False)),
                               "N": cfg.net.N, "fitness": cfg.ga.fitness,
                               "fitness_window": cfg.ga.window_for(cfg.envs_per_path),
                               "ga": not args.no_ga, "same_path": args.same_path, "dtype": tr.compute_dtype,
                               "deterministic": bool(cfg.deterministic), "lr_anneal": cfg.a2c.lr_anneal,
                               "max_time_step": cfg.a2c.max_time_step}})
        out["config"]["seed"] = cfg.seed
        if cfg.paths_total:
            out["config"]["paths_total"] = cfg.paths_total
        if build_info is not None:
            out["build"] = build_info
        print(json.dumps(out), flush=True)
        if args.out:
            os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
            with open(args.out, "w") as f:
                f.write(json.dumps(out) + "\n")
    ctx.destroy()


if __name__ == "__main__":
    main()
