"""Profiling target: the configs[2] act forward (65,536 envs, 20x20, deeper bf16 net),
each layer launched REPS times by snk_dqn_time_deep_layers."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

g = snk.SnakeGame(20, 2, n_envs=65536, autoreset=True)
m = snk.DQNModel(20, 3, n_frames=2, seed=1234, deep=True)
ms = np.zeros(6, np.float64)
_lib.call("snk_dqn_time_deep_layers", m.handle, g.handle, int(os.environ.get("REPS", "3")), _lib.ptr(ms))
print("deep layers ms", ms)
