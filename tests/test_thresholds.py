"""Calibrated solve thresholds of the synthetic games (scripts/calibrate_thresholds.py -> envs/thresholds.json) and
the SpaceInvaders wave rule (CPU)."""
import json
import os
import sys

import torch

from pathnet_gym_amd.envs import registry

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_registry_uses_calibrated_thresholds():
    with open(os.path.join(ROOT, "pathnet_gym_amd", "envs", "thresholds.json")) as f:
        doc = json.load(f)
    for g, rec in doc["games"].items():
        assert rec["expert"]["mean_return"] > rec["random"]["mean_return"], g
        assert rec["random"]["mean_return"] < rec["threshold"] <= max(rec["expert"]["mean_return"], 18.0), g
        assert registry.reward_threshold(g) == rec["threshold"]
        assert registry.reward_threshold("Synth" + g + "-v0") == rec["threshold"]
        assert registry.make(g, num_envs=1).reward_threshold == rec["threshold"]
    assert registry.reward_threshold("Pong") == 18.0
    assert registry.reward_threshold("Alien-v0") == registry.REAL_ATARI_THRESHOLDS["Alien"]     # real ids unchanged


def test_space_invaders_waves_repeat():
    env = registry.make("SpaceInvaders", num_envs=2, seed=1)
    env.reset()
    env.alive[0] = False
    env.alive[0, 5, 0] = True            # one alien left in env 0
    env.fy[0] = 40
    env._commit()
    got = 0
    for _ in range(400):
        a = torch.tensor([1, 0])
        gun = env.px[0] + 3
        target = env.fx[0] + 4
        if target > gun + 1:
            a[0] = 4
        elif target < gun - 1:
            a[0] = 5
        r, d, _ = env._advance(a)
        got += int(r[0])
        if env.alive[0].all():
            break
    assert got == 5 and env.alive[0].all() and not bool(d[0])           # cleared -> a fresh wave, same episode
    assert int(env.fy[0]) == 40 and int(env.fx[0]) in (22, 23)


def test_calibration_expert_beats_random_on_breakout():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from calibrate_thresholds import EXPERTS
    tot = {}
    for policy in ("random", "expert"):
        env = registry.make("Breakout", num_envs=8, seed=3)
        env.reset()
        g = torch.Generator().manual_seed(0)
        s = 0
        for _ in range(300):
            a = torch.randint(0, 4, (8,), generator=g) if policy == "random" else EXPERTS["Breakout"](env)
            r, _, _ = env._advance(a)
            s += int(r.sum())
        tot[policy] = s / 8
    assert tot["expert"] > tot["random"] + 10, tot
