"""Profiling target: the headline training loop (4096 x 12x12 envs, 2 frames,
one B=64 update per iteration, graph-captured), ITERS iterations after the
buffer fill (default 64)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

tr = snk.Trainer(n_envs=4096, board_size=12, n_frames=2, capacity=50000, batch_size=64, epsilon=0.05,
                 epsilon_end=0.05, decay=0.0, updates_per_iter=1, seed=7)
snk.fill_buffer_(tr, graph=True)
tr.run(int(os.environ.get("ITERS", "64")), learn=True, graph=True)
_lib.call("snk_synchronize")
print("updates", tr.stats()["updates"])
