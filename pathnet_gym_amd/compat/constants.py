"""``constants.py`` names (ref constants.py:4-32), re-exported from ``config``."""
from ..config import (ACTION_SIZEZ, ACTION_SPACE_TYPE, CHECKPOINT_DIR, ENTROPY_BETA, GAMMA,  # noqa: F401
                      GRAD_NORM_CLIP, INITIAL_ALPHA_HIGH, INITIAL_ALPHA_LOG_RATE, INITIAL_ALPHA_LOW, LOCAL_T_MAX,
                      MAX_TIME_STEP, PARALLEL_SIZE, RMSP_ALPHA, RMSP_EPSILON, ROMZ, USE_LSTM, USE_PATHNET)

import time as _time

GYM_MONITOR_DIR = "./data/gym/experiment-" + str(int(_time.time()))   # constants.py:22
NUM_GPUS = 8                       # constants.py:29 (unused by the reference): one MI355X node
USE_GPU = True                     # constants.py:31 is False (CPU TF); this engine is GPU-first
