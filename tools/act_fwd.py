"""Run the 4096-env act forward a few times (profiling target)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

g = snk.SnakeGame(12, 2, n_envs=4096, autoreset=True)
m = snk.DQNModel(12, 3, n_frames=2, seed=1234)
ms = np.zeros(5, np.float64)
_lib.call("snk_dqn_time_act_layers", m.handle, g.handle, int(os.environ.get("REPS", "5")), _lib.ptr(ms))
print("act layers ms", ms)
