"""Generations-to-solve: the reference's task horizon plus a held-out confirmation of the winning path.

The reference defines no solve criterion; BASELINE.json asks for generations-to-solve on Pong.
The criterion here:

* a tournament whose winner fitness (the mean return over the path's last E episodes, GAConfig.fitness "mean")
  reaches the env's reward threshold (Pong 18) is a solve CANDIDATE;
* the candidate's path is evaluated held-out at once (algo/evaluate.py evaluate_path: ``confirm_episodes`` fresh
  envs, one episode each, the sampled policy, the same weights, the fp32 PyTorch forward).  The solve is CONFIRMED
  when that mean reaches ``confirm_threshold`` (default 17); otherwise training goes on and the candidate is logged;
* training stops at the task horizon like the reference: its worker leaves a task once
  ``global_step > MAX_TIME_STEP * (task + 1)`` (doom_pathnet.py:197,230), which is exactly where its learning-rate
  anneal reaches 0 (a3c_training_thread.py:83-87).  Here the horizon is the frame count at which this config's anneal
  (algo/optim.py anneal_lr) reaches 0, capped by steps_per_task; a run still unconfirmed there is "unsolved at
  horizon", whatever a later tournament would have said with frozen weights.

Every rank takes the same decisions: the GA mirror is replicated, the held-out mean is rank 0's (broadcast as a max
over ranks of rank 0's value), and the horizon is a frame count.
"""
from __future__ import annotations

import math
import time
from typing import Optional

import numpy as np

from ..envs.registry import reward_threshold
from .optim import anneal_lr

CRITERION = "tournament>=threshold, held-out confirmation, task horizon (v2)"


def task_horizon_frames(cfg, task_idx: int = 0, task_start: int = 0) -> int:
    """Frames task ``task_idx`` may train for (counted from its first frame ``task_start``): where this config's
    learning rate reaches 0, capped by steps_per_task (the reference: doom_pathnet.py:197 with MAX_TIME_STEP, where
    its anneal also ends, a3c_training_thread.py:83-87)."""
    a2c = cfg.a2c
    cap = int(cfg.steps_per_task)
    if a2c.lr_anneal == "per_task":
        return min(cap, int(a2c.max_time_step))
    if a2c.lr_anneal == "global":
        return max(0, min(cap, int(a2c.max_time_step) * (task_idx + 1) - int(task_start)))
    return cap


class SolveTracker:
    """Feed every UpdateStats of a PathNetTrainer to ``observe``; it returns True once the run should stop (a confirmed
    solve or the task horizon).  ``record()`` is the JSON summary."""

    def __init__(self, tr, confirm_threshold: float = 17.0, confirm_episodes: int = 64, eval_seed: Optional[int] = None,
                 max_eval_steps: int = 30000, wall_s: float = math.inf, log=None):
        self.tr = tr
        cfg = tr.cfg
        self.task = tr.task_idx
        self.env_id = cfg.tasks[self.task]
        self.threshold = reward_threshold(self.env_id)
        self.confirm_threshold = float(confirm_threshold)
        self.confirm_episodes = int(confirm_episodes)
        # held-out envs: a seed no training env of this run uses (training: cfg.seed * 7919 + task * 113)
        self.eval_seed = int(eval_seed if eval_seed is not None else 1_000_003 + 7 * cfg.seed + 131 * self.task)
        self.max_eval_steps = int(max_eval_steps)
        self.horizon = task_horizon_frames(cfg, self.task, tr.task_start_step)
        self.wall_s = wall_s
        self.log = log
        self.t0 = time.time()
        self.eval_s = 0.0
        self.best = -math.inf
        self.candidates = []          # every held-out check: generation, updates, frames, fitness, held-out mean
        self.solved = None
        self.stopped = None           # "solved" | "horizon" | "wall"

    def lr_now(self, frames: int) -> float:
        a2c = self.tr.cfg.a2c
        return anneal_lr(a2c.lr, frames, a2c.max_time_step, self.tr.task_start_step, a2c.lr_anneal)

    def frames_in_task(self) -> int:
        return int(self.tr.global_step - self.tr.task_start_step)

    def confirm(self, path: int) -> dict:
        from .evaluate import evaluate_path
        tr = self.tr
        t = time.time()
        expr = tr.pop.expressed()[path]
        ctx = tr.ctx
        if ctx.is_main or not ctx.enabled:
            ev = evaluate_path(tr.cfg.net, tr.model.store.flat, expr, self.env_id, task=tr.model.task,
                               episodes=self.confirm_episodes, seed=self.eval_seed, device=tr.device,
                               frameskip=tr.cfg.frameskip, gray=tr.cfg.gray, max_steps=self.max_eval_steps)
        else:
            ev = {"mean": -math.inf}
        m = ev["mean"] if math.isfinite(ev["mean"]) else -math.inf
        m = ctx.max_scalar(m) if ctx.enabled else m      # rank 0's mean on every rank
        ev["mean"] = m
        ev["seconds"] = round(time.time() - t, 1)
        self.eval_s += time.time() - t
        return ev

    def observe(self, st) -> bool:
        tr = self.tr
        if self.stopped is not None:
            return True
        if st.tournaments:
            self.best = max(self.best, st.best_winner)
            if st.best_winner >= self.threshold and st.winner_path >= 0:
                frames = self.frames_in_task()
                lr = float(getattr(tr, "last_lr", self.lr_now(tr.global_step)))   # the latest optimizer step's
                ev = self.confirm(st.winner_path)
                c = {"generation": int(tr.pop.generation - tr._task_gen0), "updates": int(tr.updates),
                     "frames": frames, "lr": lr, "winner_path": int(st.winner_path),
                     "winner_fitness": float(st.best_winner), "heldout_mean": ev["mean"],
                     "heldout_min": ev.get("min"), "heldout_finished": ev.get("finished"),
                     "heldout_steps": ev.get("steps"), "eval_seconds": ev["seconds"],
                     "confirmed": bool(ev["mean"] >= self.confirm_threshold and lr > 0.0)}
                self.candidates.append(c)
                if self.log:
                    self.log(c)
                if c["confirmed"]:
                    self.solved = dict(c, seconds=round(time.time() - self.t0, 1),
                                       train_seconds=round(time.time() - self.t0 - self.eval_s, 1))
                    self.stopped = "solved"
                    return True
        if self.frames_in_task() >= self.horizon:
            self.stopped = "horizon"
            return True
        if math.isfinite(self.wall_s) and tr.updates % 32 == 0 and tr.ctx.max_scalar(time.time() - self.t0) >= self.wall_s:
            self.stopped = "wall"
            return True
        return False

    def record(self) -> dict:
        tr = self.tr
        s = self.solved
        return {"criterion": CRITERION, "threshold": self.threshold, "confirm_threshold": self.confirm_threshold,
                "confirm_episodes": self.confirm_episodes, "confirm_policy": "sampled, fp32 PyTorch forward",
                "eval_seed": self.eval_seed, "horizon_frames": self.horizon, "stopped": self.stopped,
                "solved": s is not None, "generations_to_solve": s and s["generation"],
                "updates_to_solve": s and s["updates"], "frames_to_solve": s and s["frames"],
                "seconds_to_solve": s and s["seconds"], "train_seconds_to_solve": s and s["train_seconds"],
                "lr_at_solve": s and s["lr"], "heldout_mean": s and s["heldout_mean"],
                "winner_fitness": s and s["winner_fitness"],
                "best_winner_fitness": self.best if math.isfinite(self.best) else None,
                "candidates": self.candidates, "eval_seconds": round(self.eval_s, 1),
                "frames_run": self.frames_in_task(), "updates_run": int(tr.updates),
                "generations_run": int(tr.pop.generation - tr._task_gen0), "wall_s": round(time.time() - self.t0, 1)}
