#!/usr/bin/env python3
"""Continual learning across a task sequence (BASELINE config 5: Pong -> Breakout -> SpaceInvaders -> Alien).

Each task trains the population for a frame budget. At task end the winner path is frozen together with its
task-specific head. Every other parameter is then re-initialised (doom_pathnet.py:274-293). After the last
task, every task is re-evaluated greedily with its own frozen path and head. Frozen parameters are never
updated, so the earlier tasks' scores must survive the later tasks (no catastrophic forgetting).

    python scripts/continual.py --frames 25000000 [--tasks Pong,Breakout,SpaceInvaders,Alien]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tasks", default="Pong,Breakout,SpaceInvaders,Alien")
    ap.add_argument("--frames", type=int, default=25_000_000, help="agent frames per task")
    ap.add_argument("--paths", type=int, default=16)
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--tmax", type=int, default=5)
    ap.add_argument("--N", type=int, default=10)
    ap.add_argument("--eval-episodes", type=int, default=4)
    ap.add_argument("--eval-steps", type=int, default=6000)
    ap.add_argument("--out", default="gpurun_out/continual.json")
    args = ap.parse_args()
    import numpy as np
    import torch
    from pathnet_gym_amd import _build
    from pathnet_gym_amd.algo.evaluate import evaluate_model
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.models.acnet import ACPathNet
    if torch.cuda.is_available():
        _build.build()
    cfg = preset("atari4")
    cfg.tasks = [t.strip() for t in args.tasks.split(",")]
    cfg.net.num_tasks = len(cfg.tasks)
    cfg.net.per_task_heads = True
    cfg.net.N = args.N
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = args.paths, args.envs, args.tmax
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = max(1, args.paths // 16)
    cfg.steps_per_task = args.frames
    cfg.a2c.max_time_step = args.frames
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    tr = PathNetTrainer(cfg, device=dev)
    t0 = time.time()
    per_task = []
    for ti, name in enumerate(cfg.tasks):
        if ti != tr.task_idx:
            tr._start_task(ti)
        best, n = -1e9, 0
        ts = time.time()
        while tr.global_step - tr.task_start_step < args.frames:
            st = tr.update()
            n += 1
            if st.tournaments:
                best = max(best, st.best_winner)
        tr.flush()
        winner, frozen = tr.end_task()
        per_task.append({"task": name, "updates": n, "seconds": round(time.time() - ts, 1), "best_winner": best,
                         "solved_generation": tr.solved_generation.get(ti),
                         "frozen_modules": int(frozen.sum())})
        print(json.dumps(per_task[-1]), flush=True)
    # re-evaluate every task with its own frozen path + head after the whole sequence
    evals = []
    for ti, name in enumerate(cfg.tasks):
        m = ACPathNet(cfg.net, 1, dev, "torch")
        with torch.no_grad():
            m.store.flat.copy_(tr.model.store.flat.detach())
        m.set_paths(tr.task_paths[ti][None])
        m.task = ti
        r = evaluate_model(m, name, episodes=args.eval_episodes, max_steps=args.eval_steps, device=dev,
                           frameskip=cfg.frameskip, gray=cfg.gray)
        evals.append({"task": name, "greedy_return": r[0]})
        print(json.dumps(evals[-1]), flush=True)
    out = {"tasks": cfg.tasks, "frames_per_task": args.frames, "per_task": per_task, "final_eval": evals,
           "seconds": round(time.time() - t0, 1)}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps({"done": True, "seconds": out["seconds"]}))


if __name__ == "__main__":
    main()
