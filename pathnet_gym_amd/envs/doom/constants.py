"""Doom constants: button table, level settings, game variables, resolutions.

Sources: ``gym_doom/controls.md:28-77`` (43 buttons: 38 binary, 2 delta
+/-10 look/turn, 3 delta +/-100 movement), ``gym_doom/doom_env.py:21-44``
(level table: config, scenario, map, skill, allowed buttons, min / target
score), ``doom_env.py:257-285`` (22 game variables),
``wrappers/observation_space.py:9-13`` (36 ViZDoom resolutions).
"""
NUM_ACTIONS = 43
NUM_LEVELS = 9
CONFIG, SCENARIO, MAP, DIFFICULTY, ACTIONS, MIN_SCORE, TARGET_SCORE = range(7)

BUTTONS = [
    "ATTACK", "USE", "JUMP", "CROUCH", "TURN180", "ALT_ATTACK", "RELOAD", "ZOOM", "SPEED", "STRAFE",
    "MOVE_RIGHT", "MOVE_LEFT", "MOVE_BACKWARD", "MOVE_FORWARD", "TURN_RIGHT", "TURN_LEFT", "LOOK_UP",
    "LOOK_DOWN", "MOVE_UP", "MOVE_DOWN", "LAND",
    "SELECT_WEAPON1", "SELECT_WEAPON2", "SELECT_WEAPON3", "SELECT_WEAPON4", "SELECT_WEAPON5",
    "SELECT_WEAPON6", "SELECT_WEAPON7", "SELECT_WEAPON8", "SELECT_WEAPON9", "SELECT_WEAPON0",
    "SELECT_NEXT_WEAPON", "SELECT_PREV_WEAPON", "DROP_SELECTED_WEAPON", "ACTIVATE_SELECTED_WEAPON",
    "SELECT_NEXT_ITEM", "SELECT_PREV_ITEM", "DROP_SELECTED_ITEM",
    "LOOK_UP_DOWN_DELTA", "TURN_LEFT_RIGHT_DELTA", "MOVE_FORWARD_BACKWARD_DELTA", "MOVE_LEFT_RIGHT_DELTA",
    "MOVE_UP_DOWN_DELTA",
]
assert len(BUTTONS) == NUM_ACTIONS

# per-button (low, high): 38 binary, 2 angle deltas, 3 speed deltas
BUTTON_RANGES = [(0, 1)] * 38 + [(-10, 10)] * 2 + [(-100, 100)] * 3

LEVEL_NAMES = ["DoomBasic", "DoomCorridor", "DoomDefendCenter", "DoomDefendLine", "DoomHealthGathering",
               "DoomMyWayHome", "DoomPredictPosition", "DoomTakeCover", "DoomDeathmatch"]

# (config, scenario wad, map, skill, allowed buttons, min score, target score)
DOOM_SETTINGS = [
    ["basic.cfg", "basic.wad", "map01", 5, [0, 10, 11], -485, 10],
    ["deadly_corridor.cfg", "deadly_corridor.wad", "", 1, [0, 10, 11, 13, 14, 15], -120, 1000],
    ["defend_the_center.cfg", "defend_the_center.wad", "", 5, [0, 14, 15], -1, 10],
    ["defend_the_line.cfg", "defend_the_line.wad", "", 5, [0, 14, 15], -1, 15],
    ["health_gathering.cfg", "health_gathering.wad", "map01", 5, [13, 14, 15], 0, 1000],
    ["my_way_home.cfg", "my_way_home.wad", "", 5, [13, 14, 15], -0.22, 0.5],
    ["predict_position.cfg", "predict_position.wad", "map01", 3, [0, 14, 15], -0.075, 0.5],
    ["take_cover.cfg", "take_cover.wad", "map01", 5, [10, 11], 0, 750],
    ["deathmatch.cfg", "deathmatch.wad", "", 5, [x for x in range(NUM_ACTIONS) if x != 33], 0, 20],
]
ALLOWED_ACTIONS = [row[ACTIONS] for row in DOOM_SETTINGS]

# ToDiscrete / ToBox named configurations (wrappers/action_space.py:52-62)
ACTION_CONFIGS = {
    "constant-7": [0, 10, 11, 13, 14, 15, 31],
    "constant-17": [0, 2, 3, 4, 6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 31, 32],
}

GAME_VARIABLES = ["KILLCOUNT", "ITEMCOUNT", "SECRETCOUNT", "FRAGCOUNT", "HEALTH", "ARMOR", "DEAD", "ON_GROUND",
                  "ATTACK_READY", "ALTATTACK_READY", "SELECTED_WEAPON", "SELECTED_WEAPON_AMMO",
                  "AMMO1", "AMMO2", "AMMO3", "AMMO4", "AMMO5", "AMMO6", "AMMO7", "AMMO8", "AMMO9", "AMMO0"]

RESOLUTIONS = ["160x120", "200x125", "200x150", "256x144", "256x160", "256x192", "320x180", "320x200",
               "320x240", "320x256", "400x225", "400x250", "400x300", "512x288", "512x320", "512x384",
               "640x360", "640x400", "640x480", "800x450", "800x500", "800x600", "1024x576", "1024x640",
               "1024x768", "1280x720", "1280x800", "1280x960", "1280x1024", "1400x787", "1400x875",
               "1400x1050", "1600x900", "1600x1000", "1600x1200", "1920x1080"]

# registry: id -> (level or "meta", max_episode_steps, reward_threshold)   (gym_doom/__init__.py:18-91)
REGISTRY = {
    "gym_doom/meta-Doom-v0": ("meta", 999999, 9000.0),
    "gym_doom/DoomBasic-v0": (0, 10000, 10.0),
    "gym_doom/DoomCorridor-v0": (1, 10000, 1000.0),
    "gym_doom/DoomDefendCenter-v0": (2, 10000, 10.0),
    "gym_doom/DoomDefendLine-v0": (3, 10000, 15.0),
    "gym_doom/DoomHealthGathering-v0": (4, 10000, 1000.0),
    "gym_doom/DoomMyWayHome-v0": (5, 10000, 0.5),
    "gym_doom/DoomPredictPosition-v0": (6, 10000, 0.5),
    "gym_doom/DoomTakeCover-v0": (7, 10000, 750.0),
    "gym_doom/DoomDeathmatch-v0": (8, 10000, 20.0),
}
META_KWARGS = {"average_over": 3, "passing_grade": 600, "min_tries_for_avg": 3}
