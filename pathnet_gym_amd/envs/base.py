"""Vectorised, device-resident environment API (Gym-compatible surface).

The reference drives one ``gym`` env per worker process through
``GameState`` (``game_state.py:21-84``): ``reset()``, ``process(a)`` (step),
``action_space.n``, seeding, reward, terminal.  Here an environment object
owns ``num_envs`` independent instances as device tensors; ``step`` takes
an action vector and auto-resets finished instances (the returned obs is the
first observation of the new episode, ``done`` is set for that step).

``step`` returns ``(obs, reward, done, info)`` with ``info['episode_return']``
holding the raw return of episodes that finished this step (0 elsewhere).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch


class Discrete:
    """Minimal ``gym.spaces.Discrete`` stand-in (gym is not installed here)."""

    def __init__(self, n: int):
        self.n = int(n)

    def contains(self, x) -> bool:
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class Box:
    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


def wang_hash(x: torch.Tensor) -> torch.Tensor:
    """32-bit Wang hash on int64 tensors (all intermediates < 2^63).

    Shared bit-for-bit with ``csrc/envs.hip`` so torch and HIP envs draw the
    same random numbers.
    """
    m = 0xFFFFFFFF
    x = x & m
    x = (x ^ 61) ^ (x >> 16)
    x = (x * 9) & m
    x = x ^ (x >> 4)
    x = (x * 0x27D4EB2D) & m
    x = x ^ (x >> 15)
    return x


def env_rand_u32(seed: torch.Tensor, env_id: torch.Tensor, counter: torch.Tensor, stream: int) -> torch.Tensor:
    """Counter-based RNG: hash(seed, env, counter, stream) -> uint32 in int64."""
    h = wang_hash(counter * 4 + stream)
    h = wang_hash(h ^ env_id)
    h = wang_hash(h ^ seed)
    return h


class VecEnv:
    num_envs: int
    num_actions: int
    obs_shape: Tuple[int, ...]
    obs_dtype: torch.dtype
    reward_threshold: float = float("inf")
    max_episode_steps: int = 0
    id: str = ""
    id_base: int = 0             # global index of instance 0 (RNG identity, see set_id_base)

    @property
    def action_space(self) -> Discrete:
        return Discrete(self.num_actions)

    def seed(self, seed: int):
        raise NotImplementedError

    def set_id_base(self, base: int):
        """Instance b draws its random numbers as global instance ``base + b`` (counter-based RNG keyed by the
        global index, torch and HIP alike).  A trainer rank that owns envs [base, base + num_envs) of a
        population therefore sees exactly the streams those envs have in a one-GPU run of the same seed: the
        trajectories do not depend on how the population is sharded.  Call before the first reset."""
        self.id_base = int(base)
        if isinstance(getattr(self, "env_id", None), torch.Tensor):
            self.env_id = torch.arange(self.num_envs, dtype=torch.int64, device=self.env_id.device) + self.id_base

    def reset(self) -> torch.Tensor:
        raise NotImplementedError

    def step(self, actions: torch.Tensor):
        raise NotImplementedError

    def reset_where(self, mask: torch.Tensor):
        """Start fresh episodes for instances where ``mask`` is set."""
        raise NotImplementedError

    def close(self):
        pass
