"""Batched bridge from host-side Gym environments to the device rollout.

The reference drives any ``gym`` env through ``GameState``
(``game_state.py:21-51``): ``gym.make(ROM)``, ``seed``, ``reset``, a 4-tuple
``step``, ``action_space.n``; actions ``>= n`` are remapped to 0 (``:38-39``);
frames go through BGR2GRAY + bilinear resize to 160x120 + /255 (``:41-50``)
and a 4-frame stack (``:66,78``); every reset plays ``randint(0, no_op_max)``
no-ops (``:57-60``, ``no_op_max`` = the task's action count,
``a3c_training_thread.py:81``).

``GymVecEnv`` does the same for N host envs at once and feeds the device:

* the N envs are stepped on the host (they are Python/C++ objects; there is
  no way around that), finished episodes are auto-reset with no-op starts,
  and the raw (unclipped) episode return is reported on the step that ends it;
* all N observations land in ONE pinned host buffer (``[N,210,160,3]`` uint8
  for Atari frames, ``[N,d]`` float32 for vector observations) and go to the
  GPU in ONE asynchronous H2D copy per step;
* Atari-shaped frames are preprocessed and pushed into the uint8 frame stack
  by the HIP kernel ``rgb_stack_push`` (``csrc/preprocess.hip``: gray + cv2
  INTER_LINEAR resize + shift-append, one launch for all N envs); the torch
  oracle ``envs/pong.py:preprocess_frames`` does it on CPU (bit-identical).

Both the classic API (``reset() -> obs``, ``step -> (obs, r, done, info)``)
and the gymnasium API (``reset() -> (obs, info)``, 5-tuple ``step``) are
accepted.  The bridge implements the VecEnv surface (``reset``/``step``) for
the torch trainer and ``step_into`` for the HIP engine; host stepping cannot
be captured in a hipGraph, so ``graph_safe`` is False and the engine launches
that update eagerly.

``PyCartPole`` is a pure-Python CartPole-v1 written against the classic gym
API (the env the bridge is tested with; gym itself is not installed here).
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from .base import Discrete, VecEnv
from .pong import OBS_H, OBS_W, SCREEN_H, SCREEN_W, linear_table, preprocess_frames, resize_tables


def _resize_tables_for(H: int, W: int) -> torch.Tensor:
    """cv2 INTER_LINEAR tables [8, 160] for an H x W source (any Atari-like frame size)."""
    if (H, W) == (SCREEN_H, SCREEN_W):
        return torch.from_numpy(resize_tables())
    t = np.zeros((8, OBS_H), np.int32)
    ry = linear_table(OBS_H, H)
    rx = linear_table(OBS_W, W)
    for i in range(4):
        t[i, :OBS_H] = ry[i]
        t[4 + i, :OBS_W] = rx[i]
    return torch.from_numpy(t)


def _reset(env, seed: Optional[int]):
    """Classic or gymnasium reset; returns the observation only."""
    if seed is not None:
        if hasattr(env, "seed"):
            try:
                env.seed(seed)
                seed = None
            except (TypeError, NotImplementedError, AttributeError):
                pass
    try:
        out = env.reset() if seed is None else env.reset(seed=seed)
    except TypeError:
        out = env.reset()
    if isinstance(out, tuple) and len(out) == 2 and isinstance(out[1], dict):
        out = out[0]
    return out


def _step(env, a: int):
    out = env.step(a)
    if len(out) == 5:                       # gymnasium: terminated | truncated
        obs, r, term, trunc, info = out
        return obs, float(r), bool(term) or bool(trunc), info
    obs, r, done, info = out
    return obs, float(r), bool(done), info


class GymVecEnv(VecEnv):
    """N host gym envs as one device VecEnv (see module docstring)."""

    graph_safe = False          # host stepping: the HIP engine must not capture this env in a hipGraph

    def __init__(self, envs: Sequence, device="cpu", seed: int = 0, backend: str = "torch", gray: str = "rgb",
                 no_op_max: Optional[int] = None, env_id: str = "", **_unused):
        self.envs = list(envs)
        if not self.envs:
            raise ValueError("GymVecEnv needs at least one env")
        self.num_envs = len(self.envs)
        n = {int(e.action_space.n) for e in self.envs}
        if len(n) != 1:
            raise ValueError(f"envs disagree on action_space.n: {sorted(n)}")
        self.num_actions = n.pop()
        self.device = torch.device(device)
        self.backend = backend
        self.gray = gray
        self.id = env_id
        self.seed_int = int(seed) & 0xFFFFFFFF
        # global index of envs[0] (trainer: rank * P * E, VecEnv.set_id_base): env i is seeded with
        # seed + id_base + i and draws its no-op starts from its own RNG keyed by (seed, id_base + i), so the
        # ranks of a sharded population never replay each other's emulator seeds or no-op counts (the
        # reference gives every worker its own rand_seed, a3c_training_thread.py:81)
        self.id_base = 0
        self._make_rngs()
        first = np.asarray(_reset(self.envs[0], self._env_seed(0)))
        self.pixels = first.ndim == 3 and first.shape[-1] == 3 and first.dtype == np.uint8
        # the reference plays randint(0, no_op_max) no-ops after every reset, no_op_max = action count
        self.no_op_max = (self.num_actions if self.pixels else 0) if no_op_max is None else int(no_op_max)
        pin = self.device.type == "cuda"
        if self.pixels:
            self.src_hw = first.shape[:2]
            self.obs_shape = (OBS_H, OBS_W, 4)
            self.obs_dtype = torch.uint8
            self._host = torch.empty((self.num_envs,) + first.shape, dtype=torch.uint8, pin_memory=pin)
            self.tables = _resize_tables_for(*self.src_hw).to(self.device)
            self.obs = torch.zeros(self.num_envs, OBS_H, OBS_W, 4, dtype=torch.uint8, device=self.device)
        else:
            d = int(np.prod(first.shape))
            self.obs_shape = (d,)
            self.obs_dtype = torch.float32
            self._host = torch.empty(self.num_envs, d, dtype=torch.float32, pin_memory=pin)
            self.state = torch.zeros(self.num_envs, d, device=self.device)
        self._dev = torch.empty(self._host.shape, dtype=self._host.dtype, device=self.device)
        self._rew = torch.empty(self.num_envs, dtype=torch.float32, pin_memory=pin)
        self._done = torch.empty(self.num_envs, dtype=torch.uint8, pin_memory=pin)
        self._epret = torch.empty(self.num_envs, dtype=torch.float32, pin_memory=pin)
        self.ep_ret = np.zeros(self.num_envs, np.float64)
        # the pinned host buffers are refilled only after the previous step's async copies have drained
        self._ev = torch.cuda.Event() if pin else None
        self._first = first
        self.reset()

    # -- host side ------------------------------------------------------------
    def _env_seed(self, i: int) -> int:
        return (self.seed_int + self.id_base + i) & 0xFFFFFFFF

    def _make_rngs(self):
        self.rngs = [np.random.RandomState([self.seed_int, (self.id_base + i) & 0xFFFFFFFF])
                     for i in range(self.num_envs)]

    def set_id_base(self, base: int):
        """Shard this bridge as global envs [base, base + N): re-key the seeds and no-op RNGs; the next reset()
        re-seeds every env (the constructor's reset of env 0 used the unsharded seed)."""
        self.id_base = int(base)
        self._make_rngs()
        self._first = None

    def _write(self, i: int, obs):
        o = np.asarray(obs)
        if self.pixels:
            self._host[i].numpy()[...] = o
        else:
            self._host[i].numpy()[...] = o.reshape(-1).astype(np.float32)

    def _reset_env(self, i: int, seed: Optional[int] = None):
        obs = self._first if (i == 0 and self._first is not None) else _reset(self.envs[i], seed)
        if i == 0:
            self._first = None
        if self.no_op_max > 0:
            for _ in range(self.rngs[i].randint(0, self.no_op_max + 1)):      # game_state.py:57-60
                obs, _, done, _ = _step(self.envs[i], 0)
                if done:
                    obs = _reset(self.envs[i], None)
        self.ep_ret[i] = 0.0
        return obs

    def _upload(self):
        self._dev.copy_(self._host, non_blocking=True)
        self._uploaded()

    def _uploaded(self):
        if self._ev is not None:
            self._ev.record()

    def _host_ready(self):
        if self._ev is not None:
            self._ev.synchronize()

    def _push(self, obs_in: torch.Tensor, obs_out: torch.Tensor, reset: Optional[torch.Tensor]):
        """Device: preprocess the uploaded frames and shift them into the stack (reset rows re-filled)."""
        N = self.num_envs
        if self.backend == "hip" and self.device.type == "cuda" and tuple(self.src_hw) == (SCREEN_H, SCREEN_W):
            from ..ops import envs as henv
            henv.rgb_stack_push(self._dev, obs_in, obs_out, reset, self.tables, self.gray)
            return
        f = preprocess_frames(self._dev, self.tables, self.gray)                 # [N,160,120] uint8
        src = obs_in.view(N, OBS_H, OBS_W, 4)
        pushed = torch.cat([src[..., 1:], f[..., None]], dim=3)
        if reset is not None:
            fresh = f[..., None].expand(-1, -1, -1, 4)
            pushed = torch.where(reset.bool().view(N, 1, 1, 1), fresh, pushed)
        obs_out.view(N, OBS_H, OBS_W, 4).copy_(pushed)

    # -- VecEnv API -----------------------------------------------------------
    def seed(self, seed: int):
        self.seed_int = int(seed) & 0xFFFFFFFF
        self._make_rngs()

    def reset(self):
        self._host_ready()
        for i in range(self.num_envs):
            self._write(i, self._reset_env(i, self._env_seed(i)))
        self._upload()
        if self.pixels:
            allm = torch.ones(self.num_envs, dtype=torch.uint8, device=self.device)
            self._push(self.obs.view(self.num_envs, -1), self.obs.view(self.num_envs, -1), allm)
            return self.obs.clone()
        self.state.copy_(self._dev)
        return self.state.clone()

    def reset_where(self, mask):
        m = mask.detach().cpu().numpy().astype(bool)
        self._host_ready()
        for i in np.nonzero(m)[0]:
            self._write(int(i), self._reset_env(int(i)))
        self._upload()
        if self.pixels:
            self._push(self.obs.view(self.num_envs, -1), self.obs.view(self.num_envs, -1),
                       torch.from_numpy(m.astype(np.uint8)).to(self.device))
        else:
            self.state.copy_(self._dev)

    def _host_step(self, actions: torch.Tensor):
        a = actions.detach().to("cpu", torch.int64).numpy()
        self._host_ready()
        rew, done, epret = self._rew.numpy(), self._done.numpy(), self._epret.numpy()
        for i, env in enumerate(self.envs):
            ai = int(a[i])
            if ai >= self.num_actions or ai < 0:                  # game_state.py:38-39
                ai = 0
            obs, r, d, _ = _step(env, ai)
            self.ep_ret[i] += r
            rew[i] = r
            done[i] = d
            epret[i] = self.ep_ret[i] if d else 0.0
            if d:
                obs = self._reset_env(i)
            self._write(i, obs)
        self._upload()

    def step(self, actions: torch.Tensor):
        self._host_step(actions)
        dev = self.device
        reward = self._rew.to(dev, non_blocking=True)
        done = self._done.to(dev, non_blocking=True)
        epret = self._epret.to(dev, non_blocking=True)
        self._uploaded()
        if self.pixels:
            out = torch.empty_like(self.obs)
            self._push(self.obs.view(self.num_envs, -1), out.view(self.num_envs, -1), done)
            self.obs = out
            return out.clone(), reward, done.bool(), {"episode_return": epret}
        self.state = self._dev.clone()
        return self.state.clone(), reward, done.bool(), {"episode_return": epret}

    def step_into(self, actions, obs_in, obs_out, reward, done, epret):
        """HIP engine path: write obs slot t+1 and the reward/done/return rows of the rollout buffers."""
        self._host_step(actions)
        reward.copy_(self._rew, non_blocking=True)
        done.copy_(self._done, non_blocking=True)
        epret.copy_(self._epret, non_blocking=True)
        self._uploaded()
        N = self.num_envs
        if self.pixels:
            self._push(obs_in.reshape(N, -1), obs_out.reshape(N, -1), done)
            self.obs = obs_out.view(N, OBS_H, OBS_W, 4)
        else:
            d = self.obs_shape[0]
            obs_out.view(N, -1)[:, d:].zero_()
            obs_out.view(N, -1)[:, :d].copy_(self._dev)
            self.state = self._dev.clone()

    def close(self):
        for e in self.envs:
            c = getattr(e, "close", None)
            if c is not None:
                c()


# ---------------------------------------------------------------------------
# a pure-Python gym-API env (classic control CartPole-v1)
# ---------------------------------------------------------------------------
class PyCartPole:
    """CartPole-v1 against the classic gym API (``reset``, 4-tuple ``step``, ``seed``, ``action_space``)."""

    gravity, masscart, masspole, length, force_mag, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    theta_threshold = 12 * 2 * math.pi / 360
    x_threshold = 2.4
    max_episode_steps = 500
    reward_threshold = 475.0

    def __init__(self):
        self.action_space = Discrete(2)
        self.np_random = np.random.RandomState(0)
        self.state = None
        self.steps = 0

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def reset(self):
        self.state = self.np_random.uniform(-0.05, 0.05, size=4)
        self.steps = 0
        return self.state.astype(np.float32)

    def step(self, action):
        x, x_dot, th, th_dot = self.state
        force = self.force_mag if action == 1 else -self.force_mag
        total = self.masscart + self.masspole
        pml = self.masspole * self.length
        c, s = math.cos(th), math.sin(th)
        temp = (force + pml * th_dot * th_dot * s) / total
        th_acc = (self.gravity * s - c * temp) / (self.length * (4.0 / 3.0 - self.masspole * c * c / total))
        x_acc = temp - pml * th_acc * c / total
        x, x_dot = x + self.tau * x_dot, x_dot + self.tau * x_acc
        th, th_dot = th + self.tau * th_dot, th_dot + self.tau * th_acc
        self.state = np.array([x, x_dot, th, th_dot])
        self.steps += 1
        fell = abs(x) > self.x_threshold or abs(th) > self.theta_threshold
        done = fell or self.steps >= self.max_episode_steps
        return self.state.astype(np.float32), 1.0, bool(done), {}

    def close(self):
        pass


# ---------------------------------------------------------------------------
# registration helpers
# ---------------------------------------------------------------------------
def gym_factory(entry_point: Callable[[], object], env_id: str = ""):
    """VecEnv factory for ``envs.registry.register``: N copies of ``entry_point()`` behind one bridge."""
    def make(num_envs: int = 1, device="cpu", seed: int = 0, backend: str = "torch", **kw):
        kw.pop("frameskip", None)             # the gym env applies its own frame skip
        return GymVecEnv([entry_point() for _ in range(num_envs)], device=device, seed=seed, backend=backend,
                         env_id=env_id, **kw)
    return make


def gym_make_factory(env_id: str):
    """Factory for a real gym id: ``gym.make(env_id)`` per instance, or a clear error without gym."""
    def make(num_envs: int = 1, **kw):
        try:
            import gym
        except ImportError:
            try:
                import gymnasium as gym        # noqa: F401
            except ImportError:
                raise KeyError(
                    f"{env_id!r} is a real Gym/ALE id and needs the gym (or gymnasium) package, which is not "
                    f"installed. Use the synthetic on-device games ('SynthPong-v0', 'SynthBreakout-v0', ...), or "
                    f"register your own env class with envs.registry.register_gym_env(id, entry_point).") from None
        return gym_factory(lambda: gym.make(env_id), env_id)(num_envs=num_envs, **kw)
    return make


class PyCatch:
    """A tiny Atari-shaped game against the classic gym API: 210x160x3 uint8 RGB frames, 3 actions
    (NOOP, LEFT, RIGHT).  A ball falls from a random column; +1 when the paddle catches it, -1 when
    it is missed; an episode is ``balls`` drops.  Exercises the pixel path of the bridge (gray + resize +
    stack push) the way an ALE game would."""

    H, W = SCREEN_H, SCREEN_W
    PADDLE_W, PADDLE_Y, BALL = 24, 190, 6

    def __init__(self, balls: int = 5, speed: int = 12):
        self.action_space = Discrete(3)
        self.balls, self.speed = balls, speed
        self.np_random = np.random.RandomState(0)

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def _drop(self):
        self.bx = int(self.np_random.randint(0, self.W - self.BALL))
        self.by = 0

    def _frame(self):
        f = np.zeros((self.H, self.W, 3), np.uint8)
        f[:, :] = (30, 40, 90)
        f[self.PADDLE_Y:self.PADDLE_Y + 6, self.px:self.px + self.PADDLE_W] = (200, 180, 60)
        f[self.by:self.by + self.BALL, self.bx:self.bx + self.BALL] = (240, 240, 240)
        return f

    def reset(self):
        self.px = (self.W - self.PADDLE_W) // 2
        self.left = self.balls
        self._drop()
        return self._frame()

    def step(self, action):
        self.px = int(np.clip(self.px + (-8 if action == 1 else 8 if action == 2 else 0), 0, self.W - self.PADDLE_W))
        self.by += self.speed
        r = 0.0
        if self.by + self.BALL >= self.PADDLE_Y:
            hit = self.px - self.BALL < self.bx < self.px + self.PADDLE_W
            r = 1.0 if hit else -1.0
            self.left -= 1
            self._drop()
        return self._frame(), r, self.left <= 0, {}

    def close(self):
        pass
