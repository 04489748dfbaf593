"""``game_state.GameState`` (ref ``game_state.py:21-84``) -- implemented in ``envs/game_state.py``."""
from ..envs.game_state import GameState, preprocess_numpy  # noqa: F401
