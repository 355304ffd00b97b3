"""Block clocks of grad_update_kernel (profiling build: make -C .../csrc clocks).
usage: SNK_LIB=<repo>/laplace-dqn-snake-game_amd/libsnakehip_clk.so python tools/gu_clocks.py
Runs a 4096-env trainer (B = 64), arms the clocks, runs one more iteration and prints, per
section of the grid (conv2 / conv3 / Dense1 image blocks, the strided 'other' blocks, the
Dense2 block), when its blocks started and finished their slab sums + RMSProp (us from the
first block's start), and the tail: all blocks arrived, post-update done, next draw done."""
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
wo = 7
nb2, nb3, nbd = 9, 36 * 2, wo * wo * 4
secs = [("conv2", 0, nb2), ("conv3", nb2, nb2 + nb3), ("dense1", nb2 + nb3, nb2 + nb3 + nbd),
        ("other", nb2 + nb3 + nbd, nb2 + nb3 + nbd + 16), ("dense2", nb2 + nb3 + nbd + 16, nb2 + nb3 + nbd + 17)]
nwg = secs[-1][2]
lib.snk_gu_debug_clocks.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
assert lib.snk_gu_debug_clocks(nwg, None, 1) == 0
tr.run(1, learn=True, graph=False)
buf = np.zeros((nwg, 4), np.uint64)
assert lib.snk_gu_debug_clocks(nwg, buf.ctypes.data, 0) == 0
c = buf.astype(np.float64) / 100.0
t0 = c[:, 0].min()
out = {}
for name, a, b in secs:
    cc = c[a:b]
    out[name] = {"blocks": b - a, "start_max": float(cc[:, 0].max() - t0),
                 "work_median": float(np.median(cc[:, 1] - cc[:, 0])), "work_max": float((cc[:, 1] - cc[:, 0]).max()),
                 "done_max": float(cc[:, 1].max() - t0)}
last = int(np.argmax(c[:, 2]))
out["tail"] = {"last_block": last, "all_arrived": float(c[last, 2] - t0), "post_done": float(c[last, 3] - t0),
               "draw_done": float(c[last, 1] - t0)}
print(json.dumps(out, indent=1))
