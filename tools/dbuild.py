"""One Jacobian-Gram D build over N replay slots (profiling target).
usage: python tools/dbuild.py [N] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
g = snk.SnakeGame(12, 2, n_envs=1024, autoreset=True)
rb = snk.ReplayBuffer(n, board_size=12, n_frames=2)
act = snk.DeviceArray(1024, np.uint8)
for t in range((n + 1023) // 1024):
    snk.synth_actions_dev(g, 11 + t, act)
    snk.step_indices_dev(g, act.ptr, replay=rb)
m = snk.DQNModel(12, 3, n_frames=2, seed=1234)
G = snk.DeviceArray((n, n), np.float32)
for _ in range(reps):
    _, ms = snk.jacobian_gram(m, rb, n, out=G, host=False)
    print("D build phases ms", [round(x, 3) for x in ms], flush=True)
