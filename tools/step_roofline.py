"""Step-kernel HBM roofline at large batches (configs[2]-style: 20x20 boards).

For each (n_envs, board, frames, store) the fused step!/virtual_step(/store!)
kernel is timed with HIP events (snk_env_time_step) and its algorithmic bytes
per env-step are divided by that time.
  bytes/env-step without store: read the current board + write the new one
    (2 * pitch) + 16 B state read + 16 B written + 12 B outputs + 1 B action
  with store: + (C+1) * pitch replay frames + the older C-1 frames read + 9 B
    of replay metadata  -> (C + 4) * pitch + 57 at C = 2 (bench.py's figure)
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

PEAK = 8000.0
out = []
for n, bs, C, store in [(4096, 12, 2, True), (65536, 20, 2, False), (65536, 20, 2, True),
                        (262144, 20, 2, False), (262144, 20, 2, True), (262144, 12, 2, True)]:
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * 4, board_size=bs, n_frames=C, batch_size=64) if store else None
    act = snk.DeviceArray(n, np.uint8)
    pitch = (bs * bs + 15) // 16 * 16
    for t in range(20):   # warm the boards into play
        snk.synth_actions_dev(g, 7 + t, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    snk.synth_actions_dev(g, 99, act)
    ms = _lib.f64(0)
    _lib.call("snk_env_time_step", g.handle, rb.handle if rb else None, act.ptr, 50, ctypes.byref(ms))
    bpe = (C + 4) * pitch + 57 if store else 2 * pitch + 45
    gbs = n * bpe / (ms.value * 1e-3) / 1e9
    r = dict(n_envs=n, board=bs, frames=C, store=store, ms=ms.value, env_steps_per_s=n / (ms.value * 1e-3),
             bytes_per_env_step=bpe, GBs=gbs, frac_hbm=gbs / PEAK)
    print(json.dumps(r), flush=True)
    out.append(r)
    del g, rb, act
