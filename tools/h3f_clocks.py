"""Phase clocks of the fused act forward (conv_h3f_kernel; profiling build: make -C .../csrc clocks).
usage: SNK_LIB=<repo>/laplace-dqn-snake-game_amd/libsnakehip_clk.so python tools/h3f_clocks.py
Runs a 4096-env trainer, arms the clocks, runs one more iteration, prints per-phase
medians (us) over the kernel's 1024 workgroups and the grid's timeline."""
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
nwg = 4096 // 4
lib.snk_h3f_debug_clocks.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
assert lib.snk_h3f_debug_clocks(nwg, None, 1) == 0
tr.run(1, learn=True, graph=False)
buf = np.zeros((nwg, 8), np.uint64)
assert lib.snk_h3f_debug_clocks(nwg, buf.ctypes.data, 0) == 0
c = buf.astype(np.float64) / 100.0   # s_memrealtime: 100 MHz
t0 = c[:, 0].min()
names = ["conv1", "scales_splits", "conv2", "conv3_image_bstage", "conv3_offsets", "epilogue"]
ph = {n: c[:, i + 1] - c[:, i] for i, n in enumerate(names)}
ph["lifetime"] = c[:, 6] - c[:, 0]
ph["start_offset"] = c[:, 0] - t0
out = {k: {"median": round(float(np.median(v)), 3), "max": round(float(v.max()), 3)} for k, v in ph.items()}
out["grid_end_us"] = round(float(c[:, 6].max() - t0), 3)
st = np.sort(c[:, 0] - t0)
out["start_quartiles_us"] = [round(float(st[int(q * (nwg - 1))]), 3) for q in (0, 0.25, 0.5, 0.75, 1.0)]
print(json.dumps(out))
