"""Phase clocks of deep_front_kernel (configs[2]'s fused L0-L2; profiling build: make -C
.../csrc clocks). usage: SNK_LIB=<repo>/laplace-dqn-snake-game_amd/libsnakehip_clk.so python
tools/dfr_clocks.py. Runs the configs[2] act forward (65,536 envs, 20x20) through
snk_dqn_time_deep_layers with the clocks armed, prints wave 0's mean time per sample and phase
(us) over the workgroups (barrier waits count in the phase that ends at the barrier)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

lib = _lib.load()
g = snk.SnakeGame(20, 2, n_envs=65536, autoreset=True)
m = snk.DQNModel(20, 3, n_frames=2, seed=1234, deep=True)
ms = np.zeros(6, np.float64)
_lib.call("snk_dqn_time_deep_layers", m.handle, g.handle, 2, _lib.ptr(ms))
nwg = 4096
lib.snk_dfr_debug_clocks.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
assert lib.snk_dfr_debug_clocks(nwg, None, 1) == 0
_lib.call("snk_dqn_time_deep_layers", m.handle, g.handle, 1, _lib.ptr(ms))
buf = np.zeros((nwg, 8), np.uint64)
assert lib.snk_dfr_debug_clocks(nwg, buf.ctypes.data, 0) == 0
live = buf[:, 6] > 0
c = buf[live].astype(np.float64)
names = ["boards_barrier", "L0_barrier", "L1_offsets", "L1_epilogue_2barriers", "L2_offsets", "L2_epilogue_stores"]
per = {n: float(np.mean(c[:, i] / c[:, 6])) / 100.0 for i, n in enumerate(names)}   # ticks (10 ns) -> us per sample
out = {"workgroups": int(live.sum()), "samples_per_wg": float(np.mean(c[:, 6])), "us_per_sample": per,
       "total_us_per_sample": sum(per.values()), "front_ms": float(ms[0])}
print(json.dumps(out))
