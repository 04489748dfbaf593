"""Doom environments (reference ``gym_doom/``), engine-gated.

Everything that is pure logic is implemented and unit-tested here: the
43-button action table (``controls.md``), the 9-level settings table
(``doom_env.py:33-44``), the action-space adapters (``wrappers/*.py``), the
resolution list, the MetaDoom curriculum scorer (``doom_env.py:288-454``),
the process-wide init lock (``doom_env.py:47-56``) and the registry ids
with their step limits / reward thresholds (``gym_doom/__init__.py:18-91``).

Stepping a real Doom level needs the ViZDoom engine (``vizdoom`` or the old
``doom_py``), which is not installed in this image; ``DoomEnv`` raises
``DependencyNotInstalled`` on construction without it.  The scenario ``.cfg``
files are engine data: point ``PATHNET_DOOM_ASSETS`` at a directory holding
them (names in ``DOOM_SETTINGS``).
"""
from .constants import (ACTIONS, ALLOWED_ACTIONS, BUTTONS, CONFIG, DIFFICULTY, DOOM_SETTINGS, GAME_VARIABLES,
                        MAP, MIN_SCORE, NUM_ACTIONS, NUM_LEVELS, RESOLUTIONS, SCENARIO, TARGET_SCORE, LEVEL_NAMES)
from .spaces import Box, BoxToMultiDiscrete, Discrete, DiscreteToMultiDiscrete, MultiDiscrete
from .wrappers import CustomGame, SetPlayingMode, SetResolution, ToBox, ToDiscrete, Wrapper
from .scoring import MetaDoomScorer
from .env import DependencyNotInstalled, DoomEnv, DoomLock, MetaDoomEnv, DOOM_REGISTRY, make_doom
from . import scoreboard
