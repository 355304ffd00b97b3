"""Phase clocks of the fused update forward (profiling build: make -C .../csrc clocks).
usage: SNK_LIB=<repo>/laplace-dqn-snake-game_amd/libsnakehip_clk.so python tools/upd_clocks.py
Runs a 4096-env trainer, arms the clocks, runs one more iteration, prints per-phase
medians (us) over the update forward's 256 workgroups."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

lib = _lib.load()
tr = snk.Trainer(n_batches=10, n_envs=4096, board_size=12, n_frames=2, capacity=50000, epsilon=0.05, seed=5)
snk.fill_buffer_(tr, graph=False)
tr.run(4, learn=True, graph=False)
nwg = 2 * 64 * 2
lib.snk_upd_debug_clocks.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
assert lib.snk_upd_debug_clocks(nwg, None, 1) == 0
tr.run(1, learn=True, graph=False)
buf = np.zeros((nwg, 8), np.uint64)
assert lib.snk_upd_debug_clocks(nwg, buf.ctypes.data, 0) == 0
c = buf.astype(np.float64) / 100.0
t0 = c[:, 0].min()
ph = {"phase0_loads": c[:, 1] - c[:, 0], "phase1_conv1": c[:, 2] - c[:, 1], "phase2_conv2": c[:, 3] - c[:, 2],
      "phase3_conv3": c[:, 4] - c[:, 3], "phase4_dense1": c[:, 5] - c[:, 4], "start_offset": c[:, 0] - t0,
      "lifetime": c[:, 5] - c[:, 0]}
last = buf[:, 6] > 0
if last.any():
    ph["phase5_heads_last"] = c[last, 6] - c[last, 5]
out = {k: {"median": float(np.median(v)), "max": float(v.max())} for k, v in ph.items()}
out["grid_end_us"] = float(np.max(np.where(buf[:, 6] > 0, c[:, 6], c[:, 5])) - t0)
print(json.dumps(out))
