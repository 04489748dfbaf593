"""Episode monitor for vectorised envs: the counterpart of gym's ``wrappers.Monitor``.

The reference wraps its single gym env in ``gym.wrappers.Monitor(env, GYM_MONITOR_DIR-ROM)``
when ``display=True`` (``game_state.py:29-30``, ``constants.py:22``). That writes, per
episode, the length, the reward and a timestamp to
``openaigym.episode_batch.<n>.<pid>.stats.json``, records videos on a cubic schedule, and
lists the files in ``openaigym.manifest.<n>.<pid>.manifest.json``.

``VecMonitor`` provides the same files for a ``VecEnv`` of any width:

* One record per finished episode of any instance. Each record has the length, the
  reward, a timestamp and the instance id (``episode_env``, an extension).
* Videos are raw frame dumps (``.npz``, uint8 [T, H, W]) of instance 0, the newest
  stack plane of each step. ffmpeg is not part of the image. The gym schedule is kept:
  episodes k**3 below 1000, then every 1000th.

Stats flush every ``flush_every`` episodes and on ``close()``. ``step`` needs one
host sync per call for the done mask, so the monitor is for evaluation and debug runs.
The training engine keeps its episode counters on the GPU and writes aggregated
per-update records instead (``Trainer(monitor_dir=...)``).
"""
from __future__ import annotations

import json
import os
import time
from typing import Callable, List, Optional

import numpy as np
import torch

from .base import VecEnv

_instances = 0


def capped_cubic_video_schedule(episode_id: int) -> bool:
    """gym.wrappers.monitor.capped_cubic_video_schedule."""
    if episode_id < 1000:
        return int(round(episode_id ** (1.0 / 3))) ** 3 == episode_id
    return episode_id % 1000 == 0


class VecMonitor(VecEnv):
    def __init__(self, env: VecEnv, directory: str, video_callable: Optional[Callable[[int], bool]] = None,
                 force: bool = False, flush_every: int = 100, record_video: bool = True):
        global _instances
        self.env = env
        self.num_envs, self.num_actions = env.num_envs, env.num_actions
        self.obs_shape, self.obs_dtype = env.obs_shape, env.obs_dtype
        self.reward_threshold, self.max_episode_steps = env.reward_threshold, env.max_episode_steps
        self.id = getattr(env, "id", "")
        self.directory = directory
        os.makedirs(directory, exist_ok=True)
        if force:
            for f in os.listdir(directory):
                if f.startswith("openaigym."):
                    os.remove(os.path.join(directory, f))
        self.video_callable = video_callable or capped_cubic_video_schedule
        self.record_video = record_video and len(env.obs_shape) == 3
        self.flush_every = flush_every
        self._uid = f"{_instances}.{os.getpid()}"
        _instances += 1
        self.stats_path = os.path.join(directory, f"openaigym.episode_batch.{self._uid}.stats.json")
        self.manifest_path = os.path.join(directory, f"openaigym.manifest.{self._uid}.manifest.json")
        self.initial_reset_timestamp: Optional[float] = None
        self.episode_lengths: List[int] = []
        self.episode_rewards: List[float] = []
        self.episode_env: List[int] = []
        self.timestamps: List[float] = []
        self.videos: List[List[str]] = []
        self._ret = np.zeros(env.num_envs, np.float64)
        self._len = np.zeros(env.num_envs, np.int64)
        self._frames: List[np.ndarray] = []
        self._video_episode = -1          # env 0's episode index being recorded, -1 = none
        self._env0_episodes = 0
        self._unflushed = 0

    # -- VecEnv API ------------------------------------------------------------
    @property
    def device(self):
        return getattr(self.env, "device", torch.device("cpu"))

    def seed(self, seed: int):
        return self.env.seed(seed)

    def reset(self) -> torch.Tensor:
        obs = self.env.reset()
        if self.initial_reset_timestamp is None:
            self.initial_reset_timestamp = time.time()
        self._ret[:] = 0
        self._len[:] = 0
        self._start_video(obs)
        return obs

    def reset_where(self, mask: torch.Tensor):
        self.env.reset_where(mask)
        m = mask.detach().cpu().numpy().astype(bool)
        self._ret[m] = 0
        self._len[m] = 0

    def step(self, actions: torch.Tensor):
        obs, reward, done, info = self.env.step(actions)
        r = reward.detach().float().cpu().numpy()
        d = done.detach().cpu().numpy().astype(bool)
        self._ret += r
        self._len += 1
        if self._video_episode >= 0:
            self._frames.append(self._plane(obs))
        now = time.time()
        for e in np.nonzero(d)[0]:
            self.episode_lengths.append(int(self._len[e]))
            self.episode_rewards.append(float(self._ret[e]))
            self.episode_env.append(int(e))
            self.timestamps.append(now)
            self._ret[e] = 0
            self._len[e] = 0
            self._unflushed += 1
        if d[0]:
            self._env0_episodes += 1
            self._finish_video()
            self._start_video(obs)
        if self._unflushed >= self.flush_every:
            self.flush()
        return obs, reward, done, info

    def close(self):
        self._finish_video()
        self.flush()
        self.env.close()

    # -- files -------------------------------------------------------------------
    def flush(self):
        with open(self.stats_path, "w") as f:
            json.dump({"initial_reset_timestamp": self.initial_reset_timestamp, "timestamps": self.timestamps,
                       "episode_lengths": self.episode_lengths, "episode_rewards": self.episode_rewards,
                       "episode_types": ["t"] * len(self.timestamps), "episode_env": self.episode_env}, f)
        with open(self.manifest_path, "w") as f:
            json.dump({"stats": os.path.basename(self.stats_path), "videos": self.videos,
                       "env_info": {"env_id": self.id, "num_envs": self.num_envs, "gym_version": None}}, f)
        self._unflushed = 0

    def _plane(self, obs: torch.Tensor) -> np.ndarray:
        o = obs[0].detach()
        o = o[..., -1] if o.dim() == 3 else o
        o = o.cpu().numpy()
        return o if o.dtype == np.uint8 else np.clip(o * 255.0 + 0.5, 0, 255).astype(np.uint8)

    def _start_video(self, obs):
        if self.record_video and self.video_callable(self._env0_episodes):
            self._video_episode = self._env0_episodes
            self._frames = [self._plane(obs)]
        else:
            self._video_episode = -1

    def _finish_video(self):
        if self._video_episode < 0 or not self._frames:
            return
        name = f"openaigym.video.{self._uid}.video{self._video_episode:06d}.npz"
        path = os.path.join(self.directory, name)
        np.savez_compressed(path, frames=np.stack(self._frames))
        meta = path[:-4] + ".meta.json"
        with open(meta, "w") as f:
            json.dump({"episode_id": self._video_episode, "frames": len(self._frames), "content_type": "npz/uint8"}, f)
        self.videos.append([name, os.path.basename(meta)])
        self._frames = []
        self._video_episode = -1


def load_results(directory: str) -> dict:
    """Merge every stats file in ``directory`` (gym.monitoring.load_results)."""
    out = {"episode_lengths": [], "episode_rewards": [], "timestamps": [], "initial_reset_timestamp": None}
    for f in sorted(os.listdir(directory)):
        if f.startswith("openaigym.episode_batch.") and f.endswith(".stats.json"):
            with open(os.path.join(directory, f)) as fh:
                s = json.load(fh)
            for k in ("episode_lengths", "episode_rewards", "timestamps"):
                out[k] += s[k]
            t0 = s.get("initial_reset_timestamp")
            if t0 is not None and (out["initial_reset_timestamp"] is None or t0 < out["initial_reset_timestamp"]):
                out["initial_reset_timestamp"] = t0
    return out


class UpdateMonitor:
    """Aggregated per-update episode records of the training engine (JSON lines)."""

    def __init__(self, directory: str, rank: int = 0):
        os.makedirs(directory, exist_ok=True)
        self.path = os.path.join(directory, f"openaigym.updates.{rank}.{os.getpid()}.jsonl")
        self._f = open(self.path, "a")
        self.t0 = time.time()

    def record(self, task: int, update: int, global_step: int, episodes: int, mean_return: float, generation: int):
        if episodes <= 0:
            return
        self._f.write(json.dumps({"t": round(time.time() - self.t0, 3), "task": task, "update": update,
                                  "global_step": global_step, "episodes": episodes,
                                  "mean_return": mean_return, "generation": generation}) + "\n")
        self._f.flush()

    def close(self):
        self._f.close()
