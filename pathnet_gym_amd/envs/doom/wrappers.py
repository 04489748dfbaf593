"""Doom wrappers (reference ``gym_doom/wrappers``), engine-independent.

Factories return a wrapper class (gym-style ``ToDiscrete('minimal')(env)``):

* ``ToDiscrete(config)`` / ``ToBox(config)`` with config in
  ``minimal`` (the level's allowed buttons), ``constant-7``, ``constant-17``,
  ``full`` (``wrappers/action_space.py:20-114``);
* ``SetResolution('WxH')`` (one of the 36 ViZDoom resolutions);
* ``SetPlayingMode('algo' | 'human')``;
* ``CustomGame()`` deadly-corridor customisation with the 6-button discrete
  space (``wrappers/custom_game.py:14-68``).
"""
from __future__ import annotations

from .constants import ACTION_CONFIGS, ALLOWED_ACTIONS, BUTTON_RANGES, RESOLUTIONS
from .spaces import Box, BoxToMultiDiscrete, DiscreteToMultiDiscrete, MultiDiscrete, SpaceError


class Wrapper:
    def __init__(self, env):
        self.env = env
        self.action_space = getattr(env, "action_space", None)
        self.observation_space = getattr(env, "observation_space", None)

    @property
    def unwrapped(self):
        return self.env.unwrapped if hasattr(self.env, "unwrapped") else self.env

    def step(self, action):
        return self.env.step(action)

    def reset(self):
        return self.env.reset()

    def close(self):
        return self.env.close()

    def __getattr__(self, name):
        return getattr(self.env, name)


def _allowed(config, level):
    if config == "minimal":
        return ALLOWED_ACTIONS[level]
    if config in ACTION_CONFIGS:
        return list(ACTION_CONFIGS[config])
    if config == "full":
        return None
    raise SpaceError('Invalid configuration. Valid options are "minimal", "constant-7", "constant-17", "full"')


def ToDiscrete(config: str):
    class ToDiscreteWrapper(Wrapper):
        def __init__(self, env):
            super().__init__(env)
            self.action_space = DiscreteToMultiDiscrete(self.unwrapped.action_space,
                                                        _allowed(config, self.unwrapped.level))

        def step(self, action):
            return self.env.step(self.action_space(action))
    return ToDiscreteWrapper


def ToBox(config: str):
    class ToBoxWrapper(Wrapper):
        def __init__(self, env):
            super().__init__(env)
            opts = _allowed(config, self.unwrapped.level)
            self.action_space = BoxToMultiDiscrete(self.unwrapped.action_space, opts)

        def step(self, action):
            return self.env.step(self.action_space(action))
    return ToBoxWrapper


def SetResolution(target: str):
    class SetResolutionWrapper(Wrapper):
        def __init__(self, env):
            super().__init__(env)
            if target not in RESOLUTIONS:
                raise SpaceError(f'The specified resolution "{target}" is not supported by Vizdoom.')
            w, h = (int(x) for x in target.lower().split("x"))
            u = self.unwrapped
            u.screen_width, u.screen_height = w, h
            u.screen_resolution = f"RES_{w}X{h}"
            u.observation_space = Box(0, 255, (h, w, 3))
            self.observation_space = u.observation_space
    return SetResolutionWrapper


def SetPlayingMode(mode: str):
    class SetPlayingModeWrapper(Wrapper):
        def __init__(self, env):
            super().__init__(env)
            if mode not in ("algo", "human"):
                raise SpaceError(f'The mode "{mode}" is not supported. Supported options are "algo" or "human"')
            self.unwrapped._mode = mode
    return SetPlayingModeWrapper


CUSTOM_ALLOWED = [0, 10, 11, 13, 14, 15]


def CustomGame():
    class CustomGameWrapper(Wrapper):
        def __init__(self, env):
            super().__init__(env)
            u = self.unwrapped
            u.action_space = MultiDiscrete(BUTTON_RANGES)
            u.screen_height, u.screen_width = 480, 640
            u.screen_resolution = "RES_640X480"
            u.observation_space = Box(0, 255, (480, 640, 3))
            self.observation_space = u.observation_space
            u.allowed_actions = list(CUSTOM_ALLOWED)
            u.custom_level = {"config": "deadly_corridor.cfg", "scenario": "deadly_corridor.wad", "map": "",
                              "difficulty": 1}
            self.action_space = DiscreteToMultiDiscrete(u.action_space, list(CUSTOM_ALLOWED))

        def step(self, action):
            return self.unwrapped.step(self.action_space(action))
    return CustomGameWrapper
