"""Doom through the trainer, against a stub ViZDoom engine (CPU).

The reference reaches Doom as ``gym.make('gym_doom/DoomBasic-v0')`` wrapped in ``ToDiscrete`` (game_state.py:16-27,
gym_doom/wrappers/action_space.py:20-66) on top of ``DoomEnv`` (gym_doom/doom_env.py:59-285).  ViZDoom is not in this
image, so a stub ``vizdoom`` module stands in for the engine: it records every call and plays 5-tic episodes.  What
is exercised is everything on our side of the engine boundary -- registry ids, ``DoomEnv._load_level`` / ``reset`` /
``step`` (allowed-button filtering, the finished-episode zero frame), ``MetaDoomEnv`` scoring, the ToDiscrete
adapter, the batched bridge and one trainer update.  Engine parity itself stays unpinned.
"""
import os
import sys
import types

import numpy as np
import pytest
import torch

from pathnet_gym_amd.envs import registry
from pathnet_gym_amd.envs.doom.constants import ALLOWED_ACTIONS, GAME_VARIABLES, NUM_ACTIONS


class _State:
    def __init__(self, frame, game_variables):
        self.screen_buffer = frame
        self.game_variables = game_variables


class _DoomGame:
    log = []

    def __init__(self):
        self.t = 0
        self.total = 0.0
        self.finished = False
        self.inited = False
        _DoomGame.log.append(("new", None))

    def load_config(self, path):
        assert os.path.exists(path), path
        _DoomGame.log.append(("load_config", os.path.basename(path)))

    def set_doom_scenario_path(self, p):
        _DoomGame.log.append(("scenario", os.path.basename(p)))

    def set_doom_map(self, m):
        _DoomGame.log.append(("map", m))

    def set_doom_skill(self, s):
        _DoomGame.log.append(("skill", s))

    def set_window_visible(self, v):
        assert v is False

    def init(self):
        self.inited = True
        _DoomGame.log.append(("init", None))

    def set_seed(self, s):
        _DoomGame.log.append(("seed", s))

    def new_episode(self):
        assert self.inited
        self.t, self.total, self.finished = 0, 0.0, False

    def get_state(self):
        frame = np.full((480, 640, 3), (37 * self.t) % 256, np.uint8)
        frame[:, :, 1] = 200
        return _State(frame, [float(self.t)] * len(GAME_VARIABLES))

    def make_action(self, act):
        _DoomGame.log.append(("action", tuple(act)))
        r = 1.0 if any(act) else -0.25
        self.t += 1
        self.total += r
        self.finished = self.t >= 5
        return r

    def is_episode_finished(self):
        return self.finished

    def get_total_reward(self):
        return self.total

    def close(self):
        _DoomGame.log.append(("close", None))


@pytest.fixture
def stub_engine(monkeypatch):
    mod = types.ModuleType("vizdoom")
    mod.DoomGame = _DoomGame
    mod.scenarios_path = "/stub/scenarios"
    monkeypatch.setitem(sys.modules, "vizdoom", mod)
    _DoomGame.log.clear()
    return _DoomGame


def test_doom_ids_are_registered():
    ids = registry.registered()
    for name in ("gym_doom/DoomBasic-v0", "gym_doom/meta-Doom-v0", "gym_doom/DoomDeathmatch-v0"):
        assert name in ids
    assert registry.reward_threshold("gym_doom/DoomBasic-v0") == 10.0
    assert registry.legacy_synth_id("Pong-v0") == "SynthPong-v0"
    assert registry.legacy_synth_id("PongNoFrameskip-v4") == "SynthPong-v0"
    assert registry.legacy_synth_id("SynthPong-v0") is None and registry.legacy_synth_id("Pong") is None


def test_doom_without_engine_raises(monkeypatch):
    from pathnet_gym_amd.envs.doom import DependencyNotInstalled
    monkeypatch.setitem(sys.modules, "vizdoom", None)
    monkeypatch.setitem(sys.modules, "doom_py", None)
    with pytest.raises(DependencyNotInstalled):
        registry.make("gym_doom/DoomBasic-v0", num_envs=1)


def test_doom_basic_through_bridge(stub_engine):
    env = registry.make("gym_doom/DoomBasic-v0", num_envs=2, seed=3)
    allowed = ALLOWED_ACTIONS[0]
    assert env.num_actions == len(allowed) + 1 and env.pixels and env.obs.shape == (2, 160, 120, 4)
    kinds = [k for k, _ in stub_engine.log]
    assert kinds.count("init") == 2 and ("load_config", "basic.cfg") in stub_engine.log
    stub_engine.log.clear()
    total_done = 0
    for a in range(12):
        obs, rew, done, info = env.step(torch.full((2,), a % env.num_actions, dtype=torch.int32))
        total_done += int(done.sum())
        assert obs.shape == (2, 160, 120, 4) and obs.dtype == torch.uint8
    acts = [v for k, v in stub_engine.log if k == "action"]
    # DoomEnv.step sends only the level's allowed buttons; ToDiscrete action i>0 presses allowed button i-1
    assert all(len(a) == len(allowed) for a in acts)
    assert any(sum(a) == 0 for a in acts) and any(sum(a) == 1 for a in acts)
    assert total_done >= 2          # 5-tic episodes (no-op starts included) end and auto-reset


def test_meta_doom_scoring(stub_engine):
    env = registry.make("gym_doom/meta-Doom-v0", num_envs=1)
    inner = env.envs[0].unwrapped
    for _ in range(30):
        env.step(torch.ones(1, dtype=torch.int32))
    sc = inner.scorer
    assert len(sc.scores[0]) == sc.min_tries_for_avg and any(v > 0 for v in sc.scores[0])
    assert len(sc.averages()) == 9 and sc.total_reward >= 0


def test_trainer_update_on_doom(stub_engine):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("pong")
    cfg.env = "gym_doom/DoomBasic-v0"
    cfg.tasks = [cfg.env]
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 1, 3
    cfg.backend = "torch"
    cfg.use_graph = False
    cfg.net.num_actions = 18
    tr = PathNetTrainer(cfg, device="cpu")
    st = tr.update()
    assert np.isfinite(st.loss_pi) and np.isfinite(st.loss_v)
    assert sum(1 for k, _ in stub_engine.log if k == "action") >= 3 * 1 * 3
