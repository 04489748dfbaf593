#!/usr/bin/env python3
"""Continual learning across a task sequence: the reference's only experiment, generalised to K tasks.

Reference: task 1 -> freeze the last winner -> re-initialise every other parameter -> task 2
(``doom_pathnet.py:274-293``), logged as Alien -> Centipede (``aliencentipede.txt:55-93``).  BASELINE
config 5 names the 4-task suite Pong -> Breakout -> SpaceInvaders -> Alien.

Per task this records the tournament-winner curve and generations-to-solve, the frozen path, and a greedy
evaluation of the task's own frozen path + head right after the task AND again after the whole sequence.
Frozen parameters are never updated, so the two evaluations must agree (no forgetting).  ``--control``
also trains every task >= 2 from scratch with the same budget, so transfer = sequence vs scratch.

    python scripts/continual.py --tasks Pong,Breakout --frames 30000000 --control --out profiles/continual/x.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build_cfg(args, tasks):
    from pathnet_gym_amd.config import preset
    cfg = preset(args.preset)
    cfg.tasks = list(tasks)
    cfg.env = cfg.tasks[0]
    if args.paths is None:
        args.paths = cfg.paths
    if args.envs is None:
        args.envs = cfg.envs_per_path
    if args.tmax is None:
        args.tmax = cfg.a2c.t_max
    cfg.net.num_tasks = len(cfg.tasks)
    cfg.net.per_task_heads = True
    cfg.net.N = args.N
    if args.trunk_scale:
        cfg.net.trunk_scale = args.trunk_scale
    if args.lr:
        cfg.a2c.lr = args.lr
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = args.paths, args.envs, args.tmax
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = max(1, args.paths // 16)
    cfg.steps_per_task = 2 * args.frames          # task switches are driven by this script, never automatic
    cfg.a2c.max_time_step = 2 * args.frames
    cfg.a2c.lr_anneal = "none"
    cfg.seed = cfg.ga.seed = args.seed
    if args.dtype:
        cfg.compute_dtype = args.dtype
    cfg.frame_ring = bool(args.ring)
    return cfg


def greedy_eval(tr, ti, name, args, dev, sample=False, flat=None):
    """Task ti's frozen path + head on fresh envs: argmax actions, or (sample=True) the seeded sampled policy
    (a greedy Breakout policy may never press FIRE, so no episode ends).  The ``eval_episodes`` episodes run as
    that many differently seeded envs in one batch (one episode each), so an evaluation costs one episode's steps."""
    from pathnet_gym_amd.algo.evaluate import evaluate_model
    from pathnet_gym_amd.models.acnet import ACPathNet
    import numpy as np
    import torch
    n = max(1, args.eval_episodes)
    print(json.dumps({"eval": name, "task": ti, "sample": sample, "envs": n}), flush=True)   # progress heartbeat
    m = ACPathNet(tr.cfg.net, n, dev, "torch")
    with torch.no_grad():
        m.store.flat.copy_(tr.model.store.flat.detach() if flat is None else flat)
    m.set_paths(np.repeat(tr.task_paths[ti][None], n, axis=0))
    m.task = ti
    r = evaluate_model(m, name, episodes=1, max_steps=args.eval_steps, device=dev,
                       frameskip=tr.cfg.frameskip, gray=tr.cfg.gray, sample=sample)
    r = [x for x in r if math.isfinite(x)]
    return float(np.mean(r)) if r else None


def train_task(tr, ti, args, label):
    """Train task ti of the trainer for args.frames frames; returns the per-task record (curve included)."""
    if ti != tr.task_idx:
        tr._start_task(ti)
    name = tr.cfg.tasks[ti]
    from pathnet_gym_amd.envs.registry import reward_threshold
    thr = reward_threshold(name)
    best, n, ema = -math.inf, 0, None
    curve = []
    ts = time.time()
    last = ts
    solved = None
    budget = args.frames_per_task[name]
    while tr.global_step - tr.task_start_step < budget:
        if solved is not None and args.stop_after_solve is not None and \
                tr.global_step - tr.task_start_step >= solved["frames"] + args.stop_after_solve:
            break
        st = tr.update()
        n += 1
        if not math.isnan(st.mean_return):
            ema = st.mean_return if ema is None else 0.95 * ema + 0.05 * st.mean_return
        if st.tournaments:
            best = max(best, st.best_winner)
            if solved is None and st.best_winner >= thr:
                solved = dict(generation=tr.pop.generation - tr._task_gen0, frames=tr.global_step - tr.task_start_step,
                              seconds=round(time.time() - ts, 1))
        if time.time() - last >= args.report_every:
            last = time.time()
            rec = dict(run=label, task=name, t=round(last - ts, 1), frames=tr.global_step - tr.task_start_step,
                       generation=tr.pop.generation - tr._task_gen0, best_winner=best, mean_return=ema)
            curve.append(rec)
            print(json.dumps(rec), flush=True)
    tr.flush()
    return {"task": name, "updates": n, "seconds": round(time.time() - ts, 1),
            "frames": tr.global_step - tr.task_start_step, "budget": budget,
            "threshold": thr, "best_winner": best if math.isfinite(best) else None, "final_mean_return": ema, "solved": solved is not None,
            "generations_to_solve": solved and solved["generation"], "frames_to_solve": solved and solved["frames"],
            "generations": tr.pop.generation - tr._task_gen0, "curve": curve}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tasks", default="Pong,Breakout,SpaceInvaders,Alien")
    ap.add_argument("--frames", default="25000000",
                    help="agent frames per task: one number, or one per task (comma-separated)")
    ap.add_argument("--preset", default="atari4",
                    help="atari4 (FF 5-layer trunk) | reference (L=4 + LSTM 256, T=20: the reference's own network)")
    ap.add_argument("--paths", type=int, default=None, help="default: 16 (atari4), the preset's (reference)")
    ap.add_argument("--envs", type=int, default=None, help="default: 16 (atari4), the preset's (reference)")
    ap.add_argument("--tmax", type=int, default=None, help="default: 5 (atari4), the preset's (reference)")
    ap.add_argument("--N", type=int, default=4)
    ap.add_argument("--trunk-scale", default=None, choices=["M", "none"])
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--eval-episodes", type=int, default=4)
    ap.add_argument("--eval-steps", type=int, default=6000)
    ap.add_argument("--report-every", type=float, default=20.0)
    ap.add_argument("--control", action="store_true", help="also train tasks >= 2 from scratch (transfer control)")
    ap.add_argument("--stop-after-solve", type=float, default=None,
                    help="end a task this many frames after its first solving tournament (default: run the budget)")
    ap.add_argument("--control-only", action="store_true",
                    help="only the from-scratch control runs of tasks >= 2 (e.g. in a separate job)")
    ap.add_argument("--out", default="gpurun_out/continual.json")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32", "fp32x"], help="HIP engine compute dtype")
    ap.add_argument("--ring", action="store_true", help="first layer on the frame ring (the fp32x bench default)")
    ap.add_argument("--checkpoint", default=None,
                    help="continuation checkpoint written after every task (light: no frame stacks)")
    ap.add_argument("--resume", action="store_true",
                    help="continue a sequence from --checkpoint and the per-task records already in --out")
    ap.add_argument("--max-tasks", type=int, default=None,
                    help="train at most this many tasks of the sequence in this process (then --resume)")
    args = ap.parse_args()
    if args.preset == "atari4":
        args.paths = args.paths or 16
        args.envs = args.envs or 16
        args.tmax = args.tmax or 5
    import numpy as np
    import torch
    from pathnet_gym_amd import _build
    from pathnet_gym_amd.algo.ga import decode_path
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    if torch.cuda.is_available():
        _build.build()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    tasks = [t.strip() for t in args.tasks.split(",")]
    fr = [int(float(x)) for x in str(args.frames).split(",")]
    args.frames_per_task = {t: fr[min(i, len(fr) - 1)] for i, t in enumerate(tasks)}
    args.frames = max(fr)
    cfg = build_cfg(args, tasks)
    tr = None if args.control_only else PathNetTrainer(cfg, device=dev)
    t0 = time.time()
    per_task = []
    frozen_snap = []
    controls = []
    prior_s = 0.0
    if args.resume and tr is not None and args.checkpoint and os.path.exists(args.checkpoint):
        from pathnet_gym_amd.utils import checkpoint as ckpt
        ckpt.load(tr, args.checkpoint)
        with open(args.out) as f:
            old = json.load(f)
        per_task = old["per_task"]
        controls = old.get("scratch_control", [])
        prior_s = float(old.get("seconds", 0.0))
        # frozen parameters of the finished tasks as the checkpoint holds them (taken right after their freeze)
        lay = tr.model.store.layout
        flat0 = tr.model.store.flat.detach().cpu().numpy()
        for ti in range(len(per_task)):
            keep = np.zeros(lay.numel, bool)
            for s_ in lay.segments:
                if (s_.layer >= 0 and tr.task_paths[ti][s_.layer, s_.module] > 0.5) or s_.task == ti:
                    keep[s_.offset:s_.offset + s_.numel] = True
            frozen_snap.append((keep, flat0[keep].copy()))
        print(json.dumps({"resumed": args.checkpoint, "tasks_done": len(per_task), "task_idx": tr.task_idx}), flush=True)
    n_done0 = len(per_task)

    def write_out(stage):
        out = {"experiment": "continual", "reference": "doom_pathnet.py:274-293, aliencentipede.txt:55-93",
               "stage": stage, "tasks": tasks, "frames_per_task": args.frames_per_task, "n_gpus": 1,
               "config": {"preset": args.preset, "use_lstm": cfg.net.use_lstm, "L": cfg.net.L, "paths": args.paths, "envs_per_path": args.envs, "t_max": args.tmax, "N": args.N,
                          "M": cfg.net.M, "B": cfg.ga.B, "trunk_scale": cfg.net.trunk_scale, "lr": cfg.a2c.lr,
                          "per_task_heads": True, "freeze_union": cfg.ga.freeze_union, "seed": args.seed,
                          "env_reduction": cfg.a2c.env_reduction, "dtype": tr.compute_dtype if tr else None,
                          "stop_after_solve": args.stop_after_solve},
               "per_task": per_task, "scratch_control": controls, "seconds": round(time.time() - t0, 1)}
        out["seconds"] = round(prior_s + time.time() - t0, 1)
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
        return out

    for ti, name in enumerate([] if args.control_only else tasks):
        if ti < n_done0:
            continue
        if args.max_tasks is not None and ti - n_done0 >= args.max_tasks:
            print(json.dumps({"paused": True, "tasks_done": ti, "resume_with": "--resume"}), flush=True)
            return
        rec = train_task(tr, ti, args, "sequence")
        # the parameters as the task left them: end_task re-initialises everything outside the frozen paths and
        # heads, which includes the shared LSTM cell of the reference's default network (its modules are frozen,
        # its LSTM is not -- game_ac_network.py:303-521), so "after task" is evaluated on this snapshot
        flat_task_end = tr.model.store.flat.detach().clone()
        winner, frozen = tr.end_task()
        rec["frozen_path"] = [p.tolist() for p in decode_path(tr.task_paths[ti])]
        rec["frozen_modules_total"] = int(frozen.sum())
        rec["greedy_after_task"] = greedy_eval(tr, ti, name, args, dev, flat=flat_task_end)
        rec["sampled_after_task"] = greedy_eval(tr, ti, name, args, dev, sample=True, flat=flat_task_end)
        del flat_task_end
        # snapshot of this task's frozen parameters (its modules + its head) to prove they never change again
        lay = tr.model.store.layout
        keep = np.zeros(lay.numel, bool)
        for s in lay.segments:
            if (s.layer >= 0 and tr.task_paths[ti][s.layer, s.module] > 0.5) or s.task == ti:
                keep[s.offset:s.offset + s.numel] = True
        frozen_snap.append((keep, tr.model.store.flat.detach().cpu().numpy()[keep].copy()))
        per_task.append(rec)
        print(json.dumps({k: v for k, v in rec.items() if k != "curve"}), flush=True)
        write_out("sequence")
        if args.checkpoint:
            from pathnet_gym_amd.utils import checkpoint as ckpt
            ckpt.save(tr, args.checkpoint, light=True)
    flat_end = None if tr is None else tr.model.store.flat.detach().cpu().numpy()
    for ti, name in enumerate([] if args.control_only else tasks):
        keep, vals = frozen_snap[ti]
        per_task[ti]["frozen_params_bit_identical_at_end"] = bool(np.array_equal(flat_end[keep], vals))
        per_task[ti]["greedy_after_sequence"] = greedy_eval(tr, ti, name, args, dev)
        per_task[ti]["sampled_after_sequence"] = greedy_eval(tr, ti, name, args, dev, sample=True)
        a, b = per_task[ti]["greedy_after_task"], per_task[ti]["greedy_after_sequence"]
        per_task[ti]["forgetting"] = None if a is None or b is None else a - b
        print(json.dumps({"task": name, "greedy_after_task": per_task[ti]["greedy_after_task"],
                          "greedy_after_sequence": per_task[ti]["greedy_after_sequence"],
                          "sampled_after_task": per_task[ti]["sampled_after_task"],
                          "sampled_after_sequence": per_task[ti]["sampled_after_sequence"],
                          "frozen_params_bit_identical_at_end": per_task[ti]["frozen_params_bit_identical_at_end"]}),
              flush=True)
    if per_task:
        write_out("sequence+evaluation")
    if args.control or args.control_only:
        for name in tasks[1:]:
            ctr = PathNetTrainer(build_cfg(args, [name]), device=dev)
            if tr is None:
                tr = ctr
            rec = train_task(ctr, 0, args, "scratch")
            controls.append({k: v for k, v in rec.items()})
            print(json.dumps({k: v for k, v in rec.items() if k != "curve"}), flush=True)
            write_out("control")
            del ctr
            torch.cuda.empty_cache() if dev == "cuda" else None
    out = write_out("done")
    print(json.dumps({"done": True, "seconds": out["seconds"], "out": args.out}), flush=True)


if __name__ == "__main__":
    main()
