"""Profiling driver: N back-to-back launches of the fused step kernel alone.
usage: python tools/step_only.py <n_envs> <board> <store 0|1> [launches]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402
import snake_amd as snk  # noqa: E402

n, bs, store = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
snk.load()
g = snk.SnakeGame(bs, 2, n_envs=n, autoreset=True)
rb = snk.ReplayBuffer(n * 2, board_size=bs, n_frames=2, batch_size=64) if store else None
a = snk.DeviceArray(n, np.uint8)
for t in range(reps):
    snk.synth_actions_dev(g, 7 + t, a)
    snk.step_indices_dev(g, a.ptr, replay=rb)
snk.synchronize() if hasattr(snk, "synchronize") else None
print("steps", g.t)
