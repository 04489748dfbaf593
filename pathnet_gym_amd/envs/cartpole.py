"""CartPole-v1, vectorised on device.

Dynamics and constants follow the classic-control CartPole used by gym's
``CartPole-v1`` registration (Euler integrator, tau=0.02, force 10, pole
half-length 0.5, terminate at |x|>2.4 or |theta|>12 deg, 500-step limit,
reward 1 per step, reward_threshold 475).  BASELINE.json configs 1-2.

Two implementations share this class: a pure torch one (oracle, CPU) and
the fused HIP kernel ``cartpole_step`` (``csrc/envs.hip``) on GPU.  Initial
states use the same counter-based hash RNG in both so they agree bit-for-bit
up to float rounding of the dynamics.
"""
from __future__ import annotations

import math

import torch

from .base import VecEnv, env_rand_u32

GRAVITY = 9.8
MASSCART = 1.0
MASSPOLE = 0.1
TOTAL_MASS = MASSCART + MASSPOLE
LENGTH = 0.5
POLEMASS_LENGTH = MASSPOLE * LENGTH
FORCE_MAG = 10.0
TAU = 0.02
THETA_THRESHOLD = 12 * 2 * math.pi / 360
X_THRESHOLD = 2.4


class CartPoleVec(VecEnv):
    id = "CartPole-v1"
    reward_threshold = 475.0
    max_episode_steps = 500

    def __init__(self, num_envs: int, device="cpu", seed: int = 0, backend: str = "torch"):
        self.num_envs = num_envs
        self.num_actions = 2
        self.obs_shape = (4,)
        self.obs_dtype = torch.float32
        self.device = torch.device(device)
        self.backend = backend
        self.state = torch.zeros(num_envs, 4, device=self.device)
        self.steps = torch.zeros(num_envs, dtype=torch.int32, device=self.device)
        self.ep_ret = torch.zeros(num_envs, device=self.device)
        self.counter = torch.zeros(num_envs, dtype=torch.int64, device=self.device)
        self.env_id = torch.arange(num_envs, dtype=torch.int64, device=self.device)
        self.seed(seed)

    def seed(self, seed: int):
        self.seed_int = seed & 0xFFFFFFFF
        self._seed = torch.tensor(self.seed_int, dtype=torch.int64, device=self.device)
        self.counter.zero_()

    def _rand_state(self, mask):
        u = [(env_rand_u32(self._seed, self.env_id, self.counter, s) >> 8).float() * (1.0 / 16777216.0)
             for s in range(4)]
        init = torch.stack(u, 1) * 0.1 - 0.05
        self.counter += mask.long()
        return torch.where(mask[:, None], init, self.state)

    def reset(self):
        allm = torch.ones(self.num_envs, dtype=torch.bool, device=self.device)
        self.reset_where(allm)
        return self.state.clone()

    def reset_where(self, mask):
        hip_state = hasattr(self, "_steps32")
        if hip_state:
            self.steps = self._steps32.long()
            self.counter = self._ctr32.long() & 0xFFFFFFFF
        self.state = self._rand_state(mask)
        self.steps = torch.where(mask, torch.zeros_like(self.steps), self.steps)
        self.ep_ret = torch.where(mask, torch.zeros_like(self.ep_ret), self.ep_ret)
        if hip_state:
            from ..ops import envs as henv
            henv.cartpole_sync_to_device(self)

    def step(self, actions: torch.Tensor):
        if self.backend == "hip":
            from ..ops import envs as henv
            return henv.cartpole_step(self, actions)
        x, x_dot, theta, theta_dot = self.state.unbind(1)
        force = torch.where(actions.long() == 1, FORCE_MAG, -FORCE_MAG).to(self.state.dtype)
        costheta = torch.cos(theta)
        sintheta = torch.sin(theta)
        temp = (force + POLEMASS_LENGTH * theta_dot * theta_dot * sintheta) / TOTAL_MASS
        thetaacc = (GRAVITY * sintheta - costheta * temp) / (
            LENGTH * (4.0 / 3.0 - MASSPOLE * costheta * costheta / TOTAL_MASS))
        xacc = temp - POLEMASS_LENGTH * thetaacc * costheta / TOTAL_MASS
        x = x + TAU * x_dot
        x_dot = x_dot + TAU * xacc
        theta = theta + TAU * theta_dot
        theta_dot = theta_dot + TAU * thetaacc
        self.state = torch.stack([x, x_dot, theta, theta_dot], 1)
        self.steps = self.steps + 1
        fell = (x < -X_THRESHOLD) | (x > X_THRESHOLD) | (theta < -THETA_THRESHOLD) | (theta > THETA_THRESHOLD)
        done = fell | (self.steps >= self.max_episode_steps)
        reward = torch.ones(self.num_envs, device=self.device)
        self.ep_ret = self.ep_ret + reward
        ep_return = torch.where(done, self.ep_ret, torch.zeros_like(self.ep_ret))
        self.reset_where(done)
        return self.state.clone(), reward, done, {"episode_return": ep_return}
