"""Environment registry (``make``), mirroring gym ids where they exist.

Reference tasks are gym Atari ids (``constants.py:14``) and the gym_doom
ids (``gym_doom/__init__.py:18-91``).  On-device implementations exist for
CartPole and the synthetic Atari-style games; Doom ids resolve to the
``envs/doom`` package, which needs the ViZDoom engine (not installed) for
stepping but whose action/scoring logic is pure Python.
"""
from __future__ import annotations

from typing import Callable, Dict

from .base import VecEnv

_REGISTRY: Dict[str, Callable[..., VecEnv]] = {}
_THRESHOLDS: Dict[str, float] = {}


def register(env_id: str, factory: Callable[..., VecEnv], reward_threshold: float = float("inf")):
    _REGISTRY[env_id] = factory
    _THRESHOLDS[env_id] = reward_threshold


def registered():
    return sorted(_REGISTRY)


def make(env_id: str, num_envs: int = 1, device="cpu", seed: int = 0, backend: str = "torch", **kw) -> VecEnv:
    if env_id not in _REGISTRY:
        raise KeyError(f"unknown env id {env_id!r}; registered: {registered()}")
    env = _REGISTRY[env_id](num_envs=num_envs, device=device, seed=seed, backend=backend, **kw)
    env.id = env_id
    return env


def reward_threshold(env_id: str) -> float:
    return _THRESHOLDS.get(env_id, float("inf"))


def _pong(**kw):
    from .pong import PongVec
    return PongVec(**kw)


def _cartpole(**kw):
    from .cartpole import CartPoleVec
    kw.pop("frameskip", None)
    kw.pop("gray", None)
    return CartPoleVec(**kw)


def _atari_game(name):
    def f(**kw):
        from .atari_games import make_game
        return make_game(name, **kw)
    return f


register("CartPole-v1", _cartpole, 475.0)
for _id in ("Pong", "Pong-v0", "PongNoFrameskip-v4", "PongSynth-v0"):
    register(_id, _pong, 18.0)
for _g, _thr in (("Breakout", 30.0), ("SpaceInvaders", 300.0), ("Alien", 400.0), ("MsPacman", 500.0),
                 ("Centipede", 3000.0)):
    register(_g, _atari_game(_g), _thr)
    register(_g + "-v0", _atari_game(_g), _thr)
