"""Phase clocks of conv3's and conv2's backward (profiling build: make -C .../csrc clocks).
usage: SNK_LIB=<repo>/laplace-dqn-snake-game_amd/libsnakehip_clk.so python tools/c3b_clocks.py
Runs a 4096-env trainer (B = 64 updates), arms the clocks, runs one more
iteration and prints per-phase medians (us) of the weight-gradient and the
data-gradient blocks, their start offsets (dispatch rounds) and how many
blocks shared a CU."""
import ctypes
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

lib = _lib.load()
tr = snk.Trainer(n_batches=10, n_envs=4096, board_size=12, n_frames=2, capacity=50000, epsilon=0.05, seed=5)
snk.fill_buffer_(tr, graph=False)
tr.run(4, learn=True, graph=False)
B, wo = 64, 7
nW = (B + 1) // 2 * 8
nwg = nW + B * 8
nwg2 = B + 2 * B
for f in (lib.snk_c3b_debug_clocks, lib.snk_c2b_debug_clocks):
    f.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
assert lib.snk_c3b_debug_clocks(nwg, None, 1) == 0
assert lib.snk_c2b_debug_clocks(nwg2, None, 1) == 0
tr.run(1, learn=True, graph=False)
buf = np.zeros((nwg, 8), np.uint64)
assert lib.snk_c3b_debug_clocks(nwg, buf.ctypes.data, 0) == 0
buf2 = np.zeros((nwg2, 8), np.uint64)
assert lib.snk_c2b_debug_clocks(nwg2, buf2.ctypes.data, 0) == 0
c = buf[:, :5].astype(np.float64) / 100.0
t0 = c[:, 0].min()
out = {"grid_end_us": float(c[:, 4].max() - t0), "n_wg": nwg}


def stats(v):
    return {"median": float(np.median(v)), "max": float(v.max()), "min": float(v.min()),
            "p90": float(np.percentile(v, 90)), "p97": float(np.percentile(v, 97))}


nX = B * 8   # data-gradient blocks come first in the grid
for name, sl, phases in (("dW", slice(nX, nwg), ("stage", "mfma", "store")),
                         ("dX", slice(0, nX), ("stage", "mfma", "t_store", "col2im"))):
    cc = c[sl]
    d = {"start_offset": stats(cc[:, 0] - t0), "lifetime": stats(cc[:, 4] - cc[:, 0]),
         "end": stats(cc[:, 4] - t0)}
    edges = [0, 1, 2, 3, 4] if name == "dX" else [0, 1, 2, 4]
    for k, p in enumerate(phases):
        d[p] = stats(cc[:, edges[k + 1]] - cc[:, edges[k]])
    out[name] = d
hw = buf[:, 7].astype(np.int64) - 1
xcc = buf[:, 6].astype(np.int64) - 1
cu = (xcc << 16) | ((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15)
cnt = Counter(cu.tolist())
out["distinct_cus"] = len(cnt)
out["blocks_per_cu_hist"] = dict(Counter(cnt.values()))
# concurrency: max blocks resident on one CU at any time
ev = []
for i in range(nwg):
    ev.append((c[i, 0], 1, int(cu[i])))
    ev.append((c[i, 4], -1, int(cu[i])))
ev.sort()
cur, peak = Counter(), 0
for _, dlt, k in ev:
    cur[k] += dlt
    peak = max(peak, cur[k])
out["max_resident_per_cu"] = peak
# blocks that started after the first dispatch round, and the end times of the blocks that
# shared a CU with one of them
late = c[:, 0] - t0 > 2.0
late_cus = set(cu[late].tolist())
shared = np.array([k in late_cus for k in cu.tolist()]) & ~late
out["late_blocks"] = {"n": int(late.sum()), "dW": int(late[nX:].sum()),
                      "end_of_cu_sharers": stats(c[shared, 4] - t0) if shared.any() else None,
                      "end_of_others": stats(c[~shared & ~late, 4] - t0)}
c2 = buf2[:, :5].astype(np.float64) / 100.0
t2 = c2[:, 0].min()
c2o = {"grid_end_us": float(c2[:, 4].max() - t2)}
for name, sl in (("dW", slice(0, B)), ("dX", slice(B, nwg2))):
    cc = c2[sl]
    c2o[name] = {"start_offset": stats(cc[:, 0] - t2), "lifetime": stats(cc[:, 4] - cc[:, 0]),
                 "stage": stats(cc[:, 1] - cc[:, 0]), "mfma": stats(cc[:, 2] - cc[:, 1]),
                 "epilogue": stats(cc[:, 4] - cc[:, 2])}
out["conv2_bwd"] = c2o
print(json.dumps(out, indent=1))
