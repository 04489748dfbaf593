"""Engine-backed Doom envs (reference ``gym_doom/doom_env.py``) + registry.

``DoomEnv(level)`` drives a ViZDoom game: 43-button MultiDiscrete action
space, RGB observations, buttons outside the level's allowed set are
dropped before ``make_action``, an engine that stopped returns a zero frame
with ``done=True`` (``doom_env.py:179-205``), game variables go to ``info``.
Initialisation is serialised by a process-wide lock because concurrent
ViZDoom launches crash (``DoomLock``, ``doom_env.py:47-56``; the crash log in
``vizdoom-crash.log``).  The engine (``vizdoom`` / ``doom_py``) is not part of
this image: construction raises ``DependencyNotInstalled``.
"""
from __future__ import annotations

import multiprocessing
import os

import numpy as np

from .constants import (ACTIONS, BUTTON_RANGES, CONFIG, DIFFICULTY, DOOM_SETTINGS, GAME_VARIABLES, MAP,
                        META_KWARGS, NUM_ACTIONS, REGISTRY, SCENARIO)
from .scoring import MetaDoomScorer
from .spaces import Box, MultiDiscrete


class DependencyNotInstalled(ImportError):
    pass


class DoomLock:
    """Process-wide singleton lock around engine init (doom_env.py:47-56)."""
    _instance = None

    def __init__(self):
        if DoomLock._instance is None:
            DoomLock._instance = multiprocessing.Lock()

    def get_lock(self):
        return DoomLock._instance


def _engine():
    try:
        import vizdoom as vzd      # modern package
        return vzd
    except ImportError:
        pass
    try:
        import doom_py as vzd      # the reference's 2017 package
        return vzd
    except ImportError as e:
        raise DependencyNotInstalled(
            f"{e}. Doom needs the ViZDoom engine (pip install vizdoom); it is not available in this image") from e


class DoomEnv:
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 35}

    def __init__(self, level: int, assets_dir: str = None):
        self.vzd = _engine()
        self.level = level
        self.previous_level = -1
        if not assets_dir:
            from .scenarios import assets_dir as _default_assets
            assets_dir = _default_assets()      # PATHNET_DOOM_ASSETS, or the nine generated scenario configs
        self.assets_dir = assets_dir
        self.lock = DoomLock().get_lock()
        self.action_space = MultiDiscrete(BUTTON_RANGES)
        self.allowed_actions = list(range(NUM_ACTIONS))
        self.screen_height, self.screen_width = 480, 640
        self.screen_resolution = "RES_640X480"
        self.observation_space = Box(0, 255, (480, 640, 3))
        self._mode = "algo"
        self.game = None
        self.is_initialized = False
        self.curr_seed = 0

    @property
    def unwrapped(self):
        return self

    def _load_level(self):
        vzd = self.vzd
        if self.game is not None:
            self.game.close()
        self.game = vzd.DoomGame()
        row = DOOM_SETTINGS[self.level]
        custom = getattr(self, "custom_level", None)
        cfg = custom["config"] if custom else row[CONFIG]
        self.game.load_config(os.path.join(self.assets_dir, cfg))
        scen = custom["scenario"] if custom else row[SCENARIO]
        if hasattr(vzd, "scenarios_path"):
            self.game.set_doom_scenario_path(os.path.join(vzd.scenarios_path, scen))
        mp = custom["map"] if custom else row[MAP]
        if mp:
            self.game.set_doom_map(mp)
        self.game.set_doom_skill(custom["difficulty"] if custom else row[DIFFICULTY])
        if not custom:
            self.allowed_actions = row[ACTIONS]
        self.game.set_window_visible(self._mode == "human")
        with self.lock:
            self.game.init()
        self.is_initialized = True
        self.previous_level = self.level

    def reset(self):
        if not self.is_initialized or self.previous_level != self.level:
            self._load_level()
        if self.curr_seed > 0:
            self.game.set_seed(self.curr_seed)
            self.curr_seed = 0
        self.game.new_episode()
        return self.game.get_state().screen_buffer

    def step(self, action):
        if len(action) != NUM_ACTIONS:
            action = list(action) + [0] * (NUM_ACTIONS - len(action))
        act = [int(action[i]) for i in self.allowed_actions] if self.allowed_actions else [int(x) for x in action]
        try:
            r = self.game.make_action(act)
            if self.game.is_episode_finished():
                return np.zeros(self.observation_space.shape, np.uint8), r, True, {}
            st = self.game.get_state()
            info = dict(zip(GAME_VARIABLES, list(st.game_variables)))
            info["LEVEL"] = self.level
            info["TOTAL_REWARD"] = round(self.game.get_total_reward(), 4)
            return st.screen_buffer, r, False, info
        except Exception:           # engine stopped (ViZDoomIsNotRunningException)
            return np.zeros(self.observation_space.shape, np.uint8), 0, True, {}

    def seed(self, seed=None):
        self.curr_seed = (hash(seed) if seed is not None else 0) % 2 ** 32
        return [self.curr_seed]

    def close(self):
        if self.game is not None:
            self.game.close()


class MetaDoomEnv(DoomEnv):
    def __init__(self, average_over=10, passing_grade=600, min_tries_for_avg=5, assets_dir=None):
        super().__init__(0, assets_dir)
        self.scorer = MetaDoomScorer(average_over, passing_grade, min_tries_for_avg)
        self.find_new_level = False

    def reset(self):
        if self.find_new_level:
            self.level = self.scorer.change_level()
            self.find_new_level = False
        self.scorer.level = self.level
        self.scorer.start_episode()
        return super().reset()

    def step(self, action):
        obs, _, done, info = super().step(action)
        reward = self.scorer.on_step(self.game.get_total_reward(), done)
        info["SCORES"] = self.scorer.averages()
        info["TOTAL_REWARD"] = round(self.scorer.total_reward, 4)
        info["LOCKED_LEVELS"] = list(self.scorer.locked_levels)
        if done:
            self.find_new_level = True
        return obs, reward, done, info


DOOM_REGISTRY = dict(REGISTRY)


def make_doom(env_id: str, **kw):
    if env_id not in DOOM_REGISTRY:
        raise KeyError(env_id)
    level, max_steps, thr = DOOM_REGISTRY[env_id]
    if level == "meta":
        env = MetaDoomEnv(**{**META_KWARGS, **kw})
    else:
        env = DoomEnv(level, **kw)
    env.max_episode_steps = max_steps
    env.reward_threshold = thr
    return env
