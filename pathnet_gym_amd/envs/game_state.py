"""Reference-compatible single-env adapter (``game_state.py:21-84``).

``GameState(rand_seed, ROM, display=False, no_op_max=7, task_index=-1)``
exposes ``reset() / process(a) / update() / close_env()`` and the attributes
``s_t, s_t1, reward, terminal`` exactly like the reference: observations are
float32 [160, 120, 4] in [0, 1] (gray, bilinear resize to W=120/H=160,
4-frame stack newest last), actions >= n are remapped to 0.

Backends:
* registered on-device envs (Pong, CartPole, ...): a 1-env ``VecEnv``;
* ``gym`` ids when the ``gym`` package is importable (not in this image):
  the host-side reference pipeline (``preprocess_numpy``), including the
  random no-op start; the reference's ``time.sleep(3)`` on reset and
  ``env.render()`` every step are not reproduced;
* ``gym_doom/...`` ids: ``envs/doom`` (needs the ViZDoom engine).

``display=True`` (or ``monitor_dir=``) wraps on-device envs in ``envs.monitor.VecMonitor``
writing to ``GYM_MONITOR_DIR-ROM``, as the reference's ``wrappers.Monitor`` (``:29-30``).
"""
from __future__ import annotations

import numpy as np
import torch

from .pong import OBS_H, OBS_W, gray_weights, linear_table


def preprocess_numpy(frame_rgb: np.ndarray, gray: str = "rgb") -> np.ndarray:
    """[H, W, 3] uint8 -> [160, 120] float32 in [0,1] (cv2-style fixed point, game_state.py:41-50)."""
    wr, wg, wb = gray_weights(gray)
    f = frame_rgb.astype(np.int64)
    g = (f[..., 0] * wr + f[..., 1] * wg + f[..., 2] * wb + 8192) >> 14
    H, W = g.shape
    ys0, ys1, cy0, cy1 = linear_table(OBS_H, H)
    xs0, xs1, cx0, cx1 = linear_table(OBS_W, W)
    a = g[ys0][:, xs0] * cx0 + g[ys0][:, xs1] * cx1
    b = g[ys1][:, xs0] * cx0 + g[ys1][:, xs1] * cx1
    out = (a * cy0[:, None] + b * cy1[:, None] + (1 << 21)) >> 22
    return np.clip(out, 0, 255).astype(np.float32) * (1.0 / 255.0)


class GameState:
    def __init__(self, rand_seed: int, ROM: str, display: bool = False, no_op_max: int = 7, task_index: int = -1,
                 device="cpu", gray: str = "rgb", monitor_dir=None):
        self.task_index = task_index
        self.ROM = ROM
        self.display = display
        self._no_op_max = no_op_max
        self.gray = gray
        self._vec = None
        self._gym = None
        self.rng = np.random.RandomState(rand_seed)
        from .registry import registered, make
        if ROM in registered():
            kw = {} if ROM.startswith("CartPole") else dict(no_op_max=no_op_max)
            self._vec = make(ROM, num_envs=1, device=device, seed=rand_seed, **kw)
            if display or monitor_dir:      # game_state.py:29-30: Monitor to GYM_MONITOR_DIR-ROM when displaying
                from .monitor import VecMonitor
                if monitor_dir is None:
                    from ..compat.constants import GYM_MONITOR_DIR
                    monitor_dir = GYM_MONITOR_DIR + "-" + ROM
                self._vec = VecMonitor(self._vec, monitor_dir, force=True)
            self.n_actions = self._vec.num_actions
        elif ROM.startswith("gym_doom/"):
            from .doom import make_doom
            self._gym = make_doom(ROM)
            self.n_actions = len(self._gym.allowed_actions) + 1
        else:
            try:
                import gym  # noqa: F401
            except ImportError as e:
                raise KeyError(f"{ROM!r} is neither a registered on-device env nor available through gym ({e})")
            import gym
            self._gym = gym.make(ROM)
            self._gym.seed(rand_seed)
            self.n_actions = self._gym.action_space.n
        self.reset()

    # -- reference API --------------------------------------------------------
    def _frame_from_gym(self, action):
        if action >= self.n_actions:          # game_state.py:38-39
            action = 0
        obs, reward, terminal, info = self._gym.step(action)
        return reward, terminal, preprocess_numpy(np.asarray(obs), self.gray)

    def reset(self):
        if self._vec is not None:
            obs = self._vec.reset()
            self.s_t = self._to_float(obs)
        else:
            self._gym.reset()
            for _ in range(self.rng.randint(0, self._no_op_max + 1)):     # random no-op start
                self._gym.step(0)
            _, _, x = self._frame_from_gym(0)
            self.s_t = np.stack([x, x, x, x], axis=2)
        self.reward = 0
        self.terminal = False

    def process(self, action: int):
        if self._vec is not None:
            a = torch.tensor([int(action)], device=self._vec.device)
            obs, r, d, info = self._vec.step(a)
            self.reward = float(r[0])
            self.terminal = bool(d[0])
            self.s_t1 = self._to_float(obs)
        else:
            r, t, x1 = self._frame_from_gym(action)
            self.reward, self.terminal = r, t
            self.s_t1 = np.append(self.s_t[:, :, 1:], x1[:, :, None], axis=2)

    def update(self):
        self.s_t = self.s_t1

    def close_env(self):
        if self._vec is not None:
            self._vec.close()
        else:
            self._gym.close()

    @staticmethod
    def _to_float(obs):
        o = obs[0].cpu().numpy()
        return o.astype(np.float32) * (1.0 / 255.0) if o.dtype == np.uint8 else o.astype(np.float32)
