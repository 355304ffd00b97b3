"""Phase clocks of the step kernel (profiling build: make -C .../csrc clocks).
usage: SNK_LIB=<repo>/laplace-dqn-snake-game_amd/libsnakehip_clk.so python tools/step_clocks.py <n> <bs> <store>
Per workgroup: start, scalar loads issued, boards in LDS (barrier A), logic done
(barrier B), wave 1 ticket returned, phase C stores drained (wave 0, wave 1).
Prints per-phase medians (us) and the spread of start / end times over the grid."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402
import snake_amd as snk  # noqa: E402
from snake_amd import _lib  # noqa: E402

n, bs, store = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
lib = _lib.load()
g = snk.SnakeGame(bs, 2, n_envs=n, autoreset=True)
rb = snk.ReplayBuffer(n * 2, board_size=bs, n_frames=2, batch_size=64) if store else None
a = snk.DeviceArray(n, np.uint8)
for t in range(20):
    snk.synth_actions_dev(g, 7 + t, a)
    snk.step_indices_dev(g, a.ptr, replay=rb)
nwg = (n + 63) // 64
buf = np.zeros((nwg, 8), np.uint64)
lib.snk_env_debug_clocks.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32]
rc = lib.snk_env_debug_clocks(nwg, None, 1)
assert rc == 0, lib.snk_last_error()
snk.synth_actions_dev(g, 99, a)
snk.step_indices_dev(g, a.ptr, replay=rb)
assert lib.snk_env_debug_clocks(nwg, buf.ctypes.data, 0) == 0
c = buf.astype(np.float64) / 100.0   # 100 MHz -> us
t0 = c[:, 0].min()
ph = {"scalar_issue": c[:, 1] - c[:, 0], "boards_lds": c[:, 2] - c[:, 1], "logic": c[:, 3] - c[:, 2],
      "ticket_wave1": c[:, 4] - c[:, 3], "phaseC_drain_w0": c[:, 5] - c[:, 3], "phaseC_drain_w1": c[:, 6] - c[:, 4],
      "lifetime": c[:, 5] - c[:, 0]}
out = {k: {"median": float(np.median(v)), "p90": float(np.percentile(v, 90))} for k, v in ph.items()}
out["grid_start_spread_us"] = float(c[:, 0].max() - t0)
out["grid_end_us"] = float(c[:, 5].max() - t0)
out["config"] = dict(n=n, bs=bs, store=store, workgroups=nwg)
print(json.dumps(out))
