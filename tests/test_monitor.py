"""gym-Monitor-style episode records (envs/monitor.py; reference game_state.py:29-30)."""
import json
import os

import numpy as np
import torch

from pathnet_gym_amd.envs.monitor import VecMonitor, capped_cubic_video_schedule, load_results, UpdateMonitor
from pathnet_gym_amd.envs.registry import make


def test_cubic_schedule():
    ids = [i for i in range(3000) if capped_cubic_video_schedule(i)]
    assert ids[:6] == [0, 1, 8, 27, 64, 125] and 1000 in ids and 2000 in ids and 999 not in ids


def test_vec_monitor_records_every_episode(tmp_path):
    env = make("CartPole-v1", num_envs=6, seed=3)
    mon = VecMonitor(env, str(tmp_path), flush_every=5)
    mon.reset()
    g = torch.Generator().manual_seed(0)
    ret = np.zeros(6)
    ln = np.zeros(6, np.int64)
    finished = []
    for _ in range(300):
        a = torch.randint(0, 2, (6,), generator=g)
        _, r, d, info = mon.step(a)
        ret += r.numpy()
        ln += 1
        for e in np.nonzero(d.numpy())[0]:
            finished.append((int(ln[e]), float(ret[e])))
            assert abs(float(info["episode_return"][e]) - ret[e]) < 1e-4
            ret[e] = 0
            ln[e] = 0
    mon.close()
    res = load_results(str(tmp_path))
    assert len(finished) > 10
    assert sorted(zip(res["episode_lengths"], res["episode_rewards"])) == sorted(finished)
    man = [f for f in os.listdir(tmp_path) if f.endswith(".manifest.json")]
    assert len(man) == 1
    assert json.load(open(tmp_path / man[0]))["env_info"]["num_envs"] == 6


def test_vec_monitor_video_frames(tmp_path):
    env = make("Pong", num_envs=2, seed=1)
    mon = VecMonitor(env, str(tmp_path), video_callable=lambda i: i == 0)
    obs = mon.reset()
    for _ in range(5):
        obs, *_ = mon.step(torch.zeros(2, dtype=torch.long))
    mon.close()
    vids = [f for f in os.listdir(tmp_path) if f.endswith(".npz")]
    assert len(vids) == 1
    fr = np.load(tmp_path / vids[0])["frames"]
    assert fr.shape == (6, 160, 120) and fr.dtype == np.uint8
    np.testing.assert_array_equal(fr[-1], obs[0, ..., -1].numpy())


def test_game_state_display_monitor(tmp_path):
    from pathnet_gym_amd.envs.game_state import GameState
    gs = GameState(1, "CartPole-v1", display=True, monitor_dir=str(tmp_path))
    for _ in range(200):
        gs.process(0)
        gs.update()
    gs.close_env()
    assert len(load_results(str(tmp_path))["episode_lengths"]) >= 1


def test_update_monitor(tmp_path):
    m = UpdateMonitor(str(tmp_path))
    m.record(0, 1, 100, 0, float("nan"), 0)
    m.record(0, 2, 200, 3, -20.0, 1)
    m.close()
    lines = open(m.path).read().splitlines()
    assert len(lines) == 1 and json.loads(lines[0])["episodes"] == 3
