"""Time laplace_sampling_ (la_utils.jl:97-118) at the reference's scale:
5000 sampled models, K = 58 snapshot columns, 12x12 2-frame net.
usage: python tools/lap_sampling.py [n_models] [board] [chunk]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

n_models = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 12
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 0
tr = snk.Trainer(n_envs=256, board_size=bs, n_frames=2, capacity=50000, seed=11, epsilon=0.3, epsilon_end=0.3,
                 decay=0.0)
snk.fill_buffer_(tr)
K = 58
lap = snk.LaplaceD(tr.model.P, K)
for k in range(K):           # la_utils.jl:154-158: 58 consecutive q_net snapshots while training
    tr.run(20, learn=True)
    lap.snapshot(tr.model, k)
lap.fit_center()
_lib.call("snk_synchronize")
snk.laplace_sampling_(tr, lap, n_models=min(64, n_models), seed=1, chunk=chunk)   # warm-up
_lib.call("snk_synchronize")
t0 = time.perf_counter()
res = snk.laplace_sampling_(tr, lap, n_models=n_models, seed=2, chunk=chunk)
dt = time.perf_counter() - t0
L = res["lengths"]
print(f"laplace_sampling: {n_models} models in {dt:.3f} s ({n_models / dt:.0f} models/s, "
      f"{L.sum() / dt:.0f} model-steps/s); episode length mean {L.mean():.1f} max {L.max()}, "
      f"tr_reward {res['tr_reward']:.3f}, better {res['n_better_models']}", flush=True)
