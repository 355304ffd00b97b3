"""compute_D.jl's snapshot Gram D'D at the reference's size (K = 1000 snapshots of the
12x12 net, P = 279,699) on both paths: the K-split h3 kernel (default) and the round-5
x6 slab kernel (snk.arith(syrk_ksplit=False)). Prints one JSON line per path and rep.
usage: python tools/dd_gram.py [K=1000] [reps=3]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
P = 279_699
rng = np.random.default_rng(1000)
D0 = np.cumsum(rng.standard_normal((K, P), dtype=np.float32) * np.float32(2e-4), axis=0).astype(np.float64)
D0 += rng.standard_normal(P, dtype=np.float32)[None, :] * 0.05
fl = float(K) * (K + 1) * ((P + 3) // 4 * 4)
Gs = {}
for ks in (True, False):
    with snk.arith(syrk_ksplit=ks):
        lap = snk.LaplaceD(P, K)
        for k in range(K):
            lap.set_column(k, D0[k])
        _lib.call("snk_synchronize")
        t0 = time.perf_counter()
        lap.fit_center()
        _lib.call("snk_synchronize")
        tf = time.perf_counter() - t0
        for r in range(reps):
            t0 = time.perf_counter()
            G, ms = lap.gram()
            tt = time.perf_counter() - t0
            print(json.dumps({"path": "ksplit_h3" if ks else "x6_slab", "rep": r, "fit_center_ms": 1e3 * tf,
                              "gram_kernel_ms": ms, "gram_call_ms": 1e3 * tt,
                              "tflops": fl / (ms * 1e-3) / 1e12}), flush=True)
        Gs[ks] = G
        del lap
d = np.sqrt(np.diag(Gs[False]))
print(json.dumps({"max_abs_diff_over_sqrt_gii_gjj_ksplit_vs_x6": float(np.max(np.abs(Gs[True] - Gs[False]) / np.outer(d, d)))}))
