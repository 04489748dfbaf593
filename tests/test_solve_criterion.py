"""The v2 generations-to-solve criterion (algo/solve.py): task horizon where the lr anneal ends (the reference's task
end, doom_pathnet.py:197,230 with a3c_training_thread.py:83-87) and a held-out confirmation of the winning path."""
import math

import numpy as np
import pytest
import torch

from pathnet_gym_amd.algo.evaluate import evaluate_path
from pathnet_gym_amd.algo.optim import anneal_lr
from pathnet_gym_amd.algo.solve import SolveTracker, task_horizon_frames
from pathnet_gym_amd.algo.trainer import PathNetTrainer
from pathnet_gym_amd.config import preset


def test_horizon_is_where_lr_reaches_zero():
    cfg = preset("pong")
    h = task_horizon_frames(cfg)
    assert h == cfg.a2c.max_time_step == cfg.steps_per_task
    assert anneal_lr(cfg.a2c.lr, h - 1, cfg.a2c.max_time_step) > 0.0
    assert anneal_lr(cfg.a2c.lr, h, cfg.a2c.max_time_step) == 0.0
    cfg.a2c.lr_anneal = "global"           # the reference quirk: task 2 ends at 2 x MAX_TIME_STEP in global steps
    assert task_horizon_frames(cfg, 1, task_start=cfg.a2c.max_time_step) == cfg.a2c.max_time_step
    cfg.a2c.lr_anneal = "none"
    cfg.steps_per_task = 1234
    assert task_horizon_frames(cfg) == 1234


def _trainer(steps_per_task):
    cfg = preset("cartpole-cpu")
    cfg.steps_per_task = steps_per_task
    cfg.a2c.max_time_step = steps_per_task
    cfg.a2c.lr_anneal = "per_task"
    return PathNetTrainer(cfg, device="cpu")


def test_unconfirmed_candidate_runs_to_horizon():
    tr = _trainer(4000)
    trk = SolveTracker(tr, confirm_threshold=1e9, confirm_episodes=4, max_eval_steps=600)
    trk.threshold = -math.inf              # every tournament winner is a candidate
    n = 0
    while not trk.observe(tr.update()):
        n += 1
        assert n < 1000
    rec = trk.record()
    assert rec["stopped"] == "horizon" and not rec["solved"]
    assert rec["frames_run"] >= 4000 and rec["generations_to_solve"] is None
    assert rec["candidates"] and not any(c["confirmed"] for c in rec["candidates"])
    assert all(c["lr"] > 0 and c["heldout_finished"] == 4 for c in rec["candidates"])


def test_confirmed_candidate_stops_with_lr_left():
    tr = _trainer(10 ** 6)
    trk = SolveTracker(tr, confirm_threshold=-1e9, confirm_episodes=4, max_eval_steps=600)
    trk.threshold = -math.inf
    n = 0
    while not trk.observe(tr.update()):
        n += 1
        assert n < 1000
    rec = trk.record()
    assert rec["stopped"] == "solved" and rec["solved"]
    assert rec["lr_at_solve"] > 0 and rec["generations_to_solve"] >= 1
    assert rec["updates_to_solve"] == tr.updates and rec["candidates"][-1]["confirmed"]


def test_heldout_eval_is_reproducible_and_uses_the_given_path():
    tr = _trainer(10 ** 6)
    cfg = tr.cfg
    path = tr.pop.expressed()[0]
    a = evaluate_path(cfg.net, tr.model.store.flat, path, cfg.tasks[0], episodes=6, seed=7, max_steps=600)
    b = evaluate_path(cfg.net, tr.model.store.flat, path, cfg.tasks[0], episodes=6, seed=7, max_steps=600)
    assert a["returns"] == b["returns"] and a["finished"] == 6
    # a different path (another module set) plays a different policy
    other = np.zeros_like(path)
    other[:, -1] = 1.0
    c = evaluate_path(cfg.net, tr.model.store.flat, other, cfg.tasks[0], episodes=6, seed=7, max_steps=600)
    assert c["returns"] != a["returns"]
    # the evaluated weights are a copy: the trainer's parameters are untouched
    assert tr.model.store.flat.grad is None or torch.isfinite(tr.model.store.flat.grad).all()


@pytest.mark.gpu
def test_heldout_eval_hip_env_matches_torch_env_on_gpu():
    """The held-out evaluation steps Pong in its HIP kernel on a GPU; the returns equal those of the torch game
    (same policy draws, bit-exact env)."""
    import pathnet_gym_amd.algo.evaluate as ev
    from pathnet_gym_amd import _build
    _build.build()
    cfg = preset("pong")
    from pathnet_gym_amd.models.pathnet import ParamStore
    st = ParamStore(cfg.net, "cuda", seed=3)
    path = np.zeros((cfg.net.L, cfg.net.M), np.float32)
    path[:, :4] = 1.0
    a = ev.evaluate_path(cfg.net, st.flat, path, "Pong", episodes=16, seed=11, device="cuda", max_steps=3000)
    real_make = ev.make
    try:
        ev.make = lambda *x, **k: real_make(*x, **dict(k, backend="torch"))
        b = ev.evaluate_path(cfg.net, st.flat, path, "Pong", episodes=16, seed=11, device="cuda", max_steps=3000)
    finally:
        ev.make = real_make
    assert a["finished"] == b["finished"] == 16
    assert a["returns"] == b["returns"] and a["steps"] == b["steps"]
