"""Environment registry (``make``), mirroring gym ids where they exist.

Reference tasks are gym Atari ids (``constants.py:14``) and the gym_doom
ids (``gym_doom/__init__.py:18-91``).  Three kinds of env live here:

* on-device envs: ``CartPole-v1`` (the classic-control dynamics, exact) and
  the SYNTHETIC Atari-style games ``SynthPong-v0``, ``SynthBreakout-v0``,
  ``SynthSpaceInvaders-v0``, ``SynthAlien-v0``, ``SynthMsPacman-v0``,
  ``SynthCentipede-v0`` (short aliases ``Pong``, ``Breakout``, ... are kept for
  the presets).  They are not ALE games and never answer to ALE ids;
* real Gym ids (``Pong-v0``, ``PongNoFrameskip-v4``, ``Alien-v0`` ... or any
  other id): resolved through the batched host bridge ``envs/gym_bridge.py``
  with ``gym.make`` when gym/gymnasium is importable, and a clear error
  otherwise (neither is installed in this image);
* user envs: ``register_gym_env(id, entry_point)`` puts any class with the
  classic gym API behind the same bridge.

Doom ids (``gym_doom/DoomBasic-v0`` ... ``gym_doom/meta-Doom-v0``, with the reference's step limits and
reward thresholds) resolve to ``envs/doom``: N engine-backed ``DoomEnv`` / ``MetaDoomEnv`` instances wrapped
in ``ToDiscrete('minimal')`` (the level's allowed buttons + NOOP, reference
``gym_doom/wrappers/action_space.py:20-66``) behind the batched host bridge, exactly the stack the reference
builds in ``game_state.py:16-27``.  Construction needs the ViZDoom engine (``vizdoom`` / ``doom_py``), which is
not installed in this image, and raises ``DependencyNotInstalled`` without it.

Renamed ids (breaking change of round 2): the synthetic games answered to ``Pong-v0``,
``PongNoFrameskip-v4`` and ``<Game>-v0`` in round 1; those ids now mean the REAL gym games (bridge).  The
synthetic ones are ``Synth<Game>-v0`` or the short ``<Game>`` aliases; ``legacy_synth_id`` maps an old id
found in a round-1 config/checkpoint to its synthetic equivalent.
"""
from __future__ import annotations

from typing import Callable, Dict

from .base import VecEnv

_REGISTRY: Dict[str, Callable[..., VecEnv]] = {}
_THRESHOLDS: Dict[str, float] = {}
_SYNTH_ALIASES: Dict[str, str] = {}

# real ALE ids the reference and BASELINE.json name; reward thresholds are the solve criteria used here
REAL_ATARI_THRESHOLDS = {"Pong": 18.0, "Breakout": 30.0, "SpaceInvaders": 300.0, "Alien": 400.0,
                         "MsPacman": 500.0, "Centipede": 3000.0}


def register(env_id: str, factory: Callable[..., VecEnv], reward_threshold: float = float("inf")):
    _REGISTRY[env_id] = factory
    _THRESHOLDS[env_id] = reward_threshold


def register_gym_env(env_id: str, entry_point: Callable[[], object], reward_threshold: float = float("inf")):
    """Register a class/callable that builds ONE env with the classic gym API (``reset``, ``step``,
    ``action_space.n``); ``make(env_id, num_envs=N)`` then returns N of them behind ``GymVecEnv``."""
    from .gym_bridge import gym_factory
    register(env_id, gym_factory(entry_point, env_id), reward_threshold)


def registered():
    return sorted(_REGISTRY)


def is_synthetic(env_id: str) -> bool:
    return env_id in _SYNTH_ALIASES


def make(env_id: str, num_envs: int = 1, device="cpu", seed: int = 0, backend: str = "torch", **kw) -> VecEnv:
    factory = _REGISTRY.get(env_id)
    if factory is None:
        if "/" in env_id:
            raise KeyError(f"unknown env id {env_id!r}; registered: {registered()}")
        from .gym_bridge import gym_make_factory
        factory = gym_make_factory(env_id)          # raises a clear KeyError when gym is not importable
    if not is_synthetic(env_id):
        kw.pop("frameskip", None)                   # gym envs apply their own frame skip
    env = factory(num_envs=num_envs, device=device, seed=seed, backend=backend, **kw)
    env.id = env_id
    if is_synthetic(env_id):
        env.reward_threshold = reward_threshold(env_id)     # the calibrated one (envs/thresholds.json)
    return env


def legacy_synth_id(env_id: str):
    """Round-1 id of a synthetic game (``Pong-v0``, ``PongNoFrameskip-v4``, ``Breakout-v0`` ...) -> the synthetic
    id it meant then (``SynthPong-v0`` ...), or None when ``env_id`` never named a synthetic game."""
    base = env_id.split("-")[0].replace("NoFrameskip", "").replace("Deterministic", "")
    if base in REAL_ATARI_THRESHOLDS and env_id != base and not env_id.startswith("Synth"):
        return "Synth" + base + "-v0"
    return None


def reward_threshold(env_id: str) -> float:
    if env_id in _THRESHOLDS:
        return _THRESHOLDS[env_id]
    base = env_id.split("-")[0].replace("NoFrameskip", "").replace("Deterministic", "")
    return REAL_ATARI_THRESHOLDS.get(base, float("inf"))


def _pong(**kw):
    from .pong import PongVec
    return PongVec(**kw)


def _cartpole(**kw):
    from .cartpole import CartPoleVec
    kw.pop("frameskip", None)
    kw.pop("gray", None)
    kw.pop("no_op_max", None)
    return CartPoleVec(**kw)


def _atari_game(name):
    def f(**kw):
        from .atari_games import make_game
        return make_game(name, **kw)
    return f


def synthetic_thresholds() -> Dict[str, float]:
    """Solve thresholds of the synthetic games, calibrated by ``scripts/calibrate_thresholds.py`` from a measured
    random-policy return and a scripted expert's (``envs/thresholds.json``: random + 0.75 (expert - random); Pong
    keeps the ALE 18).  Real gym ids keep ``REAL_ATARI_THRESHOLDS``."""
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "thresholds.json")
    out = dict(REAL_ATARI_THRESHOLDS)
    if os.path.exists(path):
        with open(path) as f:
            for g, rec in json.load(f)["games"].items():
                out[g] = float(rec["threshold"])
    return out


register("CartPole-v1", _cartpole, 475.0)
for _g, _thr in synthetic_thresholds().items():
    _f = _pong if _g == "Pong" else _atari_game(_g)
    for _id in ("Synth" + _g + "-v0", _g):
        register(_id, _f, _thr)
        _SYNTH_ALIASES[_id] = _g


def _doom(env_id: str):
    def f(num_envs: int = 1, device="cpu", seed: int = 0, backend: str = "torch", **kw):
        from .doom import ToDiscrete, make_doom
        from .gym_bridge import GymVecEnv
        kw.pop("frameskip", None)                   # ViZDoom tics are the env's own
        envs = [ToDiscrete("minimal")(make_doom(env_id)) for _ in range(num_envs)]
        return GymVecEnv(envs, device=device, seed=seed, backend=backend, env_id=env_id, **kw)
    return f


def _register_doom():
    from .doom.constants import REGISTRY as DOOM_IDS
    for _id, (_level, _steps, _thr) in DOOM_IDS.items():
        register(_id, _doom(_id), _thr)


_register_doom()


def _register_bridge_examples():
    from .gym_bridge import PyCartPole, PyCatch
    register_gym_env("PyCartPole-v1", PyCartPole, 475.0)
    register_gym_env("PyCatch-v0", PyCatch, 4.0)


_register_bridge_examples()
