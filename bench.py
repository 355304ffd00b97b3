#!/usr/bin/env python3
"""bench.py — throughput of the batched Snake-DQN hot path on MI355X.

Metric (BASELINE.json): env-steps/sec @4096 envs (+ D(50k) build sec).
Workload (BASELINE.json configs[1]): 4096 parallel 12x12 envs, 2-frame
3-action DQN, fp32, per GPU (weak scaling). One timed "step" is one lockstep
iteration of the whole hot path, replayed from one captured hipGraph:
  epsilon_greedy Q forward over all 4096 envs -> step!/virtual_step/auto-reset
  -> store! into the 50k replay -> one DQN update (sample 64, t_net TD target,
  Huber, backward, RMSProp, target-sync check) [-> RCCL gradient all-reduce
  for N > 1].
value = env-steps of all ranks / max-over-ranks wall time. Synthetic data:
env dynamics are the real game from SnakeGame(); the net is glorot-initialised
(no checkpoint of the 2-frame 12x12 net exists).

python bench.py [--gpus N] [--steps K] [--warmup W] [--workload configs1|configs3]
For N > 1 launch one process per GPU with torch.distributed.run. --workload
configs3 runs BASELINE configs[3]: 32,768 envs per GPU (262,144 at --gpus 8);
the default N=1 line also carries that shard on one GPU (configs3_per_rank).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
PEAK_BF16_TFLOPS = 2516.0  # MI355X_MICROARCH.md: BF16 MFMA dense peak (2.5 PF, no sparsity)
X6_PRODUCTS = 6            # bf16 MFMA products per fp32 product in the exact-split forward
H3_PRODUCTS = 3            # fp16 MFMA products per fp32 product in the h3 conv3 (snk_conv_h3.hpp)
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E spec peak
CONFIGS3_ENVS_PER_GPU = 262144 // 8   # BASELINE configs[3]: 262,144 envs sharded over 8 GPUs


def act_forward_flop(n: int, bs: int, C: int) -> float:
    """FLOP of the fused act-forward kernel (conv_h3f_kernel: conv1 + conv2 + conv3)
    over n states: 2 n (bs^2 16 9C + bs^2 32 144 + Wo^2 64 1152)."""
    wo = bs - 5
    return 2.0 * n * (bs * bs * 16 * 9 * C + bs * bs * 32 * 144 + wo * wo * 64 * 1152)


def update_flop(B: int, bs: int, C: int) -> float:
    """Algorithmic FLOP of one B-sample DQN update (BASELINE.md's DQN-update row,
    4 B F): forward of q_net and of t_net over the batch (2 F each sample) and
    the backward of q_net (2 F: dX and dW). F = the fused conv stack + Dense
    Wo^2*64 -> 64 + Dense 64 -> 3 of one state (the reference net,
    structs.jl:133-134): 9,037,184 at 12x12, C = 2, so 2,313,519,104 at B = 64."""
    wo = bs - 5
    f = act_forward_flop(1, bs, C) + 2.0 * (wo * wo * 64 * 64 + 64 * 3)
    return 4.0 * B * f


def _latest_traffic(kern: str, pattern: str = "*_conv3_traffic.json"):
    """HBM bytes per launch of a dominant kernel from the newest committed PMC pass
    (profiles/*_conv3_traffic.json for the act forward, *_syrk_traffic.json for the
    D build; written by tools/traffic.py from separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 --pmc runs of tools/pmc_traffic.sh, FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 note), for the kernel this run uses."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", pattern)), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("kernel", "").startswith(kern):
            d["source"] = os.path.relpath(f, REPO) + ": " + d.get("how", "")
            return d
    return None


def _latest_pmc(kern: str, pattern: str):
    """Counter summary (tools/pmc_summary.py over the separate counter-only passes of
    tools/pmc_any.sh / pmc_syrk.sh) of the newest committed profiles/<pattern> whose kernel
    name starts with kern: MFMA busy at the clock the chip held (GRBM_GUI_ACTIVE), that
    clock, LDS bank-conflict share, for the roofline objects."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", pattern)), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if k.startswith(kern) and "mfma_busy" in v:
                return {"pmc_kernel": k.split("(")[0], "pmc_mfma_busy_nominal_clock": v.get("mfma_busy"),
                        "pmc_clock_ghz": v.get("clock_ghz"), "pmc_mfma_busy_at_clock": v.get("mfma_busy_at_clock"),
                        "pmc_lds_bank_conflict_frac": v.get("lds_conflict_frac"),
                        "pmc_source": os.path.relpath(f, REPO)}
    return {}


class _stdout_to_stderr:
    """RCCL prints its version banner to stdout when a communicator is created; the bench's
    stdout is the one JSON line, so fd 1 points at fd 2 for the duration."""

    def __enter__(self):
        sys.stdout.flush()
        self.fd = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.fd, 1)
        os.close(self.fd)


def _update_pmc() -> dict:
    """MFMA busy (nominal clock) and LDS conflicts of the five B = 64 update kernels from the
    newest committed profiles/*_pmc_update.json (tools/pmc_round.sh over the training loop;
    microsecond dispatches carry no clock: pmc_summary.py's 0.3 ms rule)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_update.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        out = {k.split("(")[0]: {"mfma_busy_nominal_clock": v.get("mfma_busy"),
                                 "lds_bank_conflict_frac": v.get("lds_conflict_frac"),
                                 "clock_note": v.get("clock_note")}
               for k, v in d.items() if "mfma_busy" in v}
        if out:
            out["source"] = os.path.relpath(f, REPO)
            return out
    return {}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--repeats", type=int, default=5,
                   help="timed windows of --steps steps each; value and ms_per_step are the median window's")
    p.add_argument("--workload", choices=("configs1", "configs3"), default="configs1",
                   help="configs1: 4096 envs per GPU (BASELINE configs[1], the metric's workload); configs3: "
                        "32,768 envs per GPU, configs[3]'s 262,144 envs over 8 GPUs (--gpus 8)")
    p.add_argument("--n-envs", type=int, default=0, help="envs per GPU (0: the workload's)")
    p.add_argument("--board-size", type=int, default=12)
    p.add_argument("--n-frames", type=int, default=2)
    p.add_argument("--updates-per-iter", type=int, default=1)
    p.add_argument("--graph-unroll", type=int, default=8,
                   help="lockstep iterations per captured hipGraph (each graph starts with the fresh "
                        "weight splits and pays one graph launch)")
    p.add_argument("--epsilon", type=float, default=0.05)
    p.add_argument("--capacity", type=int, default=50000)
    p.add_argument("--settle-ms", type=float, default=300.0,
                   help="untimed iterations after the warm-up, for this long, before the timed windows")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip per-kernel timing")
    p.add_argument("--no-dbuild", action="store_true", help="skip the Laplace D builds")
    p.add_argument("--no-configs2", action="store_true", help="skip the configs[2] deep bf16 net line")
    p.add_argument("--no-configs3", action="store_true", help="skip the configs[3] per-rank shard line")
    p.add_argument("--d-samples", type=int, default=0, help="Jacobian Gram rows (0 = the whole replay buffer)")
    p.add_argument("--d-snapshots", type=int, default=1000, help="K of the snapshot D (compute_D.jl:51)")
    p.add_argument("--arith", action="append", default=[], metavar="NAME=0|1",
                   help="A/B measurement: a non-default snk.set_arith knob (repeatable); the line's config records it")
    a = p.parse_args()
    if a.n_envs <= 0:
        a.n_envs = CONFIGS3_ENVS_PER_GPU if a.workload == "configs3" else 4096
    return a


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args) -> dict:
    """The CPU baseline: oracle/cpu_fast.cpp, an optimised
    C++ restatement of the same iteration (O(1)-collision env, fp32
    im2col + blocked GEMM Q-net and update, OpenMP), timed on this host for
    whole iterations: act forward over every env, env step + store, one B=64
    DQN update. 1 thread, then the CPU share of this job (OMP_NUM_THREADS, else
    every core). Plus the D(50k) Gram on a 2,000-row sample of Jacobian-sized
    rows, extrapolated by the n(n+1)/2 tile count (labelled)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    L = oracle.fast()
    bs, C, n = args.board_size, args.n_frames, args.n_envs
    food, _ = oracle.food_list(bs)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    t1, tn = np.zeros(4), np.zeros(4)
    v1 = L.cpuf_bench(n, bs, C, 1, 0, 1, args.updates_per_iter, args.capacity, food, len(food), t1)
    vn = L.cpuf_bench(n, bs, C, threads, 1, 3, args.updates_per_iter, args.capacity, food, len(food), tn)
    ns, Kc = 6000, 9 * C * 16 + 16 + 4640 + 73792
    X = np.random.default_rng(0).standard_normal((ns, Kc)).astype(np.float32)
    G = np.zeros((ns, ns), np.float32)
    tg = L.cpuf_gram(ns, Kc, X, G, threads)
    N = args.d_samples or 50_000
    return {"value": vn, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "sample": (f"oracle/cpu_fast.cpp (optimised C++ restatement, OpenMP, x86-64-v3): whole iterations of "
                       f"{n} envs ({bs}x{bs}, {C} frames): act forward + step/store + {args.updates_per_iter} B=64 "
                       f"update(s); {threads} threads: 3 iterations (fwd {tn[0]:.2f}s, step {tn[1]:.3f}s, "
                       f"update {tn[2]:.2f}s); 1 thread: 1 iteration (fwd {t1[0]:.2f}s, step {t1[1]:.3f}s, "
                       f"update {t1[2]:.2f}s)"),
            "cores_note": (f"the job's CPU share on the GPU box (OMP_NUM_THREADS = {threads}) of {os.cpu_count()} "
                           f"host CPUs shared with other jobs"),
            "env_steps_per_s_step_only": n * 3 / max(tn[1], 1e-12),
            "updates_per_s": 3 * args.updates_per_iter / max(tn[2], 1e-12),
            "act_forward_states_per_s": n * 3 / max(tn[0], 1e-12),
            "single_thread": {"value": v1, "cores": 1, "env_steps_per_s_step_only": n / max(t1[1], 1e-12),
                              "updates_per_s": args.updates_per_iter / max(t1[2], 1e-12)},
            "d_build_gram_sec_extrapolated": tg * (N * (N + 1.0)) / (ns * (ns + 1.0)),
            "d_build_gram_sample": f"G = X X' of {ns} rows x {Kc} conv columns in {tg:.2f}s on {threads} threads "
                                   f"({2.0 * ns * (ns + 1) / 2 * Kc / tg / 1e9:.0f} GFLOP/s), scaled by the "
                                   f"n(n+1)/2 ratio to n = {N}; Jacobian rows and the dense terms (<2% of the "
                                   f"work) not included"}


def _deep_traffic(d: int, n: int, bs: int) -> dict:
    """PMC bytes per launch of the configs[2] dominant layer (the 6x6 64->64 conv,
    deep_conv3_kernel<20>) from profiles/*_deep_traffic.json (tools/pmc_traffic.sh
    <tag> deep + tools/traffic.py), when this run's dominant layer is that one at 65,536 x 20x20."""
    if d != 3 or n != 65536 or bs != 20:
        return {}
    t = _latest_traffic("deep_conv3_kernel<20>", "*_deep_traffic.json")
    return dict(({"traffic": t["bytes_per_launch"], "traffic_source": t["source"],
                  "traffic_over_algorithmic": t["bytes_per_launch"] / t["algorithmic_bytes_per_launch"]} if t else {}),
                **_latest_pmc("deep_conv3_kernel<20>", "*_pmc_deep.json"))


def configs2(args, snk, graph) -> dict:
    """BASELINE.json configs[2]: 65,536 lockstep 20x20 envs with the deeper
    bf16 conv Q-net (snk_dqn_create_deep), one trainer
    iteration per step as the headline (act forward, step + store, one B=64
    update), median of 3 windows of 10 steps; per-layer times of the act
    forward and the roofline of its dominant kernel (bf16 MFMA peak)."""
    import numpy as np
    from snake_amd import _lib
    n, bs, C = 65536, 20, args.n_frames
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=args.capacity, batch_size=64,
                     epsilon=args.epsilon, epsilon_end=args.epsilon, decay=0.0, updates_per_iter=1, seed=4321,
                     deep=True)
    snk.fill_buffer_(tr, graph=graph)
    tr.run(2, learn=True, graph=graph)
    steps, windows = 10, []
    for _ in range(3):
        _lib.call("snk_synchronize")
        t0 = time.perf_counter()
        tr.run(steps, learn=True, graph=graph)
        _lib.call("snk_synchronize")
        windows.append(time.perf_counter() - t0)
    el = float(np.median(windows))
    ms = np.zeros(6, np.float64)
    _lib.call("snk_dqn_time_deep_layers", tr.model.handle, tr.game.handle, 5, _lib.ptr(ms))
    wo, nc = bs - 5, bs * bs
    flop = [2.0 * n * nc * 32 * 9 * C, 2.0 * n * nc * 32 * 288, 2.0 * n * nc * 64 * 288,
            2.0 * n * wo * wo * 64 * 2304, 2.0 * n * wo * wo * 64 * 64, 2.0 * n * 64 * 3]
    # L0..L2 run as one launch (deep_front_kernel): its time is ms[0], ms[1] = ms[2] = 0
    names = ["L0+L1+L2 conv 3x3 C->32->32->64 (deep_front_kernel, bf16 MFMA, fused in LDS)",
             "L1 (inside deep_front_kernel)", "L2 (inside deep_front_kernel)",
             "L3 conv 6x6 64->64 (deep_conv3_kernel, bf16 MFMA, two samples per step)",
             "Dense1 (deep_dense1_ldsb_kernel, bf16 MFMA)", "head (Dense2 + epsilon-greedy)"]
    flop = [flop[0] + flop[1] + flop[2], 0.0, 0.0] + flop[3:]
    d = int(np.argmax(ms[:5]))
    tf = flop[d] / (ms[d] * 1e-3) / 1e12
    fwd_flop = sum(flop)
    st = tr.stats()
    return {"workload": f"configs[2]: {n} lockstep {bs}x{bs} envs, {C}-frame deeper conv Q-net (bf16): eps-greedy "
                        f"forward + step!/virtual_step + store! + 1 B=64 update per step",
            "value": n * steps / el, "unit": "env-steps/s", "ms_per_step": 1000.0 * el / steps,
            "windows_ms": [1000.0 * w for w in windows], "steps": steps, "dtype": "bf16",
            "n_params": tr.model.P, "forward_flop_per_env_step": fwd_flop / n,
            "act_forward_ms": {nm: float(t) for nm, t in zip(names, ms) if t > 0},
            "act_forward_total_ms": float(ms.sum()),
            "act_forward_tflops": fwd_flop / (ms.sum() * 1e-3) / 1e12,
            "roofline": dict({"bound": "mfma", "kernel": names[d], "achieved": tf, "peak": PEAK_BF16_TFLOPS,
                              "unit": "TFLOP/s (bf16)", "frac": tf / PEAK_BF16_TFLOPS, "avg_launch_ms": float(ms[d]),
                              "flop_per_launch": flop[d], "traffic": None},
                             **_deep_traffic(d, n, bs)),
            "train_stats": {"updates": st["updates"], "episodes": st["episodes"], "env_steps": st["env_steps"]}}


def configs3_per_rank(args, snk, graph) -> dict:
    """BASELINE.json configs[3] is 262,144 lockstep envs over 8 GPUs: 32,768 per
    GPU, each rank with its own 50k replay shard and B = 64 per update (the
    ranks' mean gradient all-reduce adds one RCCL call per update at N > 1;
    bench.py --workload configs3 --gpus 8 runs the whole config). This is one
    rank's shard on this GPU: the same trainer graph as the headline at 32,768
    12x12 envs, median of 3 windows of 16 steps, and the dominant kernel's
    roofline (conv_h3f_kernel over 32,768 states, HIP events in the loop)."""
    import numpy as np
    from snake_amd import _lib
    n, bs, C = CONFIGS3_ENVS_PER_GPU, args.board_size, args.n_frames
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=args.capacity, batch_size=64,
                     epsilon=args.epsilon, epsilon_end=args.epsilon, decay=0.0, updates_per_iter=1, seed=3333)
    snk.fill_buffer_(tr, graph=graph)
    tr.run(16, learn=True, graph=graph)
    steps, windows = 16, []
    for _ in range(3):
        _lib.call("snk_synchronize")
        t0 = time.perf_counter()
        tr.run(steps, learn=True, graph=graph)
        _lib.call("snk_synchronize")
        windows.append(time.perf_counter() - t0)
    el = float(np.median(windows))
    loop_ms = _lib.f64(0)
    _lib.call("snk_trainer_time_act_kernel", tr.handle, 10, ctypes.byref(loop_ms))
    fl = act_forward_flop(n, bs, C)
    peak = PEAK_BF16_TFLOPS / H3_PRODUCTS
    tf = fl / (loop_ms.value * 1e-3) / 1e12 if loop_ms.value > 0 else 0.0
    st = tr.stats()
    return {"workload": f"configs[3] per-rank shard: {n} lockstep {bs}x{bs} envs on this GPU ({C} frames, replay "
                        f"{args.capacity}, 1 B=64 update per step) = 262,144 / 8 ranks",
            "value": n * steps / el, "unit": "env-steps/s", "ms_per_step": 1000.0 * el / steps,
            "windows_ms": [1000.0 * w for w in windows], "steps": steps,
            "effective_global_batch_at_8": 8 * 64,
            "roofline": {"bound": "mfma", "kernel": "conv_h3f_kernel (conv1 + conv2 + conv3 of the act forward)",
                         "achieved": tf, "peak": peak, "unit": "TFLOP/s (fp32-equivalent)", "frac": tf / peak,
                         "avg_launch_ms": loop_ms.value, "flop_per_launch": fl,
                         "avg_launch_ms_how": "HIP events recorded by the launch's dispatch (hipExtLaunchKernelGGL), "
                                              "median of 10 eager training iterations behind graph replays"},
            "train_stats": {"updates": st["updates"], "episodes": st["episodes"], "env_steps": st["env_steps"],
                            "food_faults": tr.game.check_faults()}}


def step_kernel_point(snk, n, bs, C, store):
    """The fused step!/virtual_step(/store!) kernel alone, back-to-back launches
    between one HIP event pair (snk_env_time_step). Algorithmic bytes per
    env-step: the current board read + the new one written (2 * pitch), 16 B
    state read + 16 B written, 12 B of step outputs, the action byte; with the
    store also b_{t-1} read and the C + 1 replay frames written + 9 B of replay
    metadata: (C + 4) * pitch + 57 at C = 2, 2 * pitch + 45 without."""
    import ctypes
    import numpy as np
    from snake_amd import _lib
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * 2, board_size=bs, n_frames=C, batch_size=64) if store else None
    a = snk.DeviceArray(n, np.uint8)
    for t in range(20):   # boards into play
        snk.synth_actions_dev(g, 7 + t, a)
        snk.step_indices_dev(g, a.ptr, replay=rb)
    snk.synth_actions_dev(g, 99, a)
    ms = _lib.f64(0)
    _lib.call("snk_env_time_step", g.handle, rb.handle if rb else None, a.ptr, 50, ctypes.byref(ms))
    pitch = (bs * bs + 15) // 16 * 16
    bpe = (C + 4) * pitch + 57 if store else 2 * pitch + 45
    gbs = n * bpe / (ms.value * 1e-3) / 1e9
    mall = n * (3 * pitch + 2 * bs * bs + 40) < 256e6
    return {"n_envs": n, "board": bs, "store": store,
            "residency": "MALL (working set < 256 MB Infinity Cache)" if mall else "HBM",
            "avg_launch_ms": ms.value, "bytes_per_env_step": bpe, "achieved_GBs": gbs,
            "frac_hbm": gbs / PEAK_HBM_GBS, "env_steps_per_s": n / (ms.value * 1e-3)}


def reference_ratio(args, snk, graph, episodes_per_env_step) -> dict:
    """The reference's own ratio of updates to play: one update per finished
    episode (utils.jl:434-481). At the headline workload about
    episodes_per_env_step x 4096 episodes end per lockstep step, so this runs
    that many B=64 updates per step: updates/s and env-steps/s of an
    update-bound loop, and the time of one update from the difference with
    the 1-update step."""
    import numpy as np
    from snake_amd import _lib
    n, bs, C = args.n_envs, args.board_size, args.n_frames
    U = max(2, int(round(episodes_per_env_step * n)))
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=args.capacity, batch_size=64,
                     epsilon=args.epsilon, epsilon_end=args.epsilon, decay=0.0, updates_per_iter=U, seed=99,
                     graph_unroll=1)
    snk.fill_buffer_(tr, graph=graph)
    tr.run(1, learn=True, graph=graph)
    steps, windows = 3, []
    for _ in range(3):
        _lib.call("snk_synchronize")
        t0 = time.perf_counter()
        tr.run(steps, learn=True, graph=graph)
        _lib.call("snk_synchronize")
        windows.append(time.perf_counter() - t0)
    el = float(np.median(windows))
    return {"updates_per_step": U, "updates_per_s": U * steps / el, "env_steps_per_s": n * steps / el,
            "ms_per_step": 1000.0 * el / steps, "ms_per_update": 1000.0 * el / steps / U}


def d_buffer(snk, bs, C, n):
    """The D(50k) replay: n transitions of lockstep play (5000 envs x n/5000
    steps, counter-RNG actions from a fixed seed). Deterministic, so every
    rank of a multi-GPU build holds the same buffer without moving it."""
    import numpy as np
    n_env = 5000 if n % 5000 == 0 else n
    g = snk.SnakeGame(bs, C, n_envs=n_env, autoreset=True)
    rb = snk.ReplayBuffer(n, board_size=bs, n_frames=C, batch_size=64)
    act = snk.DeviceArray(n_env, np.uint8)
    for _ in range(n // n_env):
        snk.synth_actions_dev(g, 0xD50, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    return rb


def d_build_gram(args, snk, model, dist, rank, world) -> dict:
    """D(50k): G = J J' over the 50,000 per-sample Jacobians of the D buffer
    (north_star / configs[4]). world > 1: each rank computes its contiguous
    run of the lower-triangle tiles (snk_jacobian_gram_shard), then rank 0
    receives the others' tiles over RCCL send/recv (snk_jacobian_gram_gather).
    d_build_sec = max-over-ranks shard time + the gather (G complete on rank 0)."""
    import time

    import numpy as np
    from snake_amd import _lib

    n = args.d_samples or 50_000
    rb = d_buffer(snk, args.board_size, args.n_frames, n)
    Kc = 9 * args.n_frames * 16 + 16 + 4640 + 73792            # conv columns of a Jacobian row
    G = snk.DeviceArray((n, n), np.float32)

    def sync():
        _lib.call("snk_synchronize")
        if dist is not None:
            dist.barrier()

    if world == 1:
        snk.jacobian_gram(model, rb, n, out=G, host=False)   # workspace allocation + first launch
        sync()
        t0 = time.perf_counter()
        _, ms = snk.jacobian_gram(model, rb, n, out=G, host=False)
        wall = time.perf_counter() - t0
        t_gather = 0.0
        gather_check = None
    else:
        import torch
        uid = snk.dist.broadcast_bytes(dist, snk.Comm.unique_id() if rank == 0 else None, rank)
        with _stdout_to_stderr():
            comm = snk.Comm(world, rank, uid)
        G.zero()
        snk.jacobian_gram_shard(model, rb, n, rank, world, G)     # warm-up
        sync()
        t0 = time.perf_counter()
        ms = snk.jacobian_gram_shard(model, rb, n, rank, world, G)
        sync()
        wall = time.perf_counter() - t0
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        t0 = time.perf_counter()
        snk.jacobian_gram_gather(comm, n, G, 0)
        sync()
        t_gather = time.perf_counter() - t0
        del comm
        gather_check = None
        if rank == 0:   # the assembled G against one whole-matrix launch on rank 0 (untimed)
            G1 = snk.DeviceArray((n, n), np.float32)
            snk.jacobian_gram(model, rb, n, out=G1, host=False)
            rows = np.sort(np.random.default_rng(7).choice(n, 16, replace=False))
            bad, dmax = 0, 0.0
            for r in rows:
                a = _lib.view_numpy(G.ptr.value + int(r) * n * 4, (n,), np.float32)
                b = _lib.view_numpy(G1.ptr.value + int(r) * n * 4, (n,), np.float32)
                bad += int(np.count_nonzero(a != b))
                dmax = max(dmax, float(np.max(np.abs(a.astype(np.float64) - b))))
            gather_check = {"rows_compared": len(rows), "entries_compared": len(rows) * n,
                            "mismatched_entries": bad, "max_abs_diff": dmax,
                            "against": "single-launch snk_jacobian_gram on rank 0 (bit-exact expected)"}
            del G1
        sync()
    T = (n + 127) // 128
    tiles = len(snk.gram_tiles(n, rank, world))
    flop_gram = float(n) * (n + 1) * Kc * tiles / (T * (T + 1) // 2)   # this rank's share, 2 flop / MAC
    tf = flop_gram / (ms[2] * 1e-3) / 1e12
    speak = PEAK_BF16_TFLOPS / H3_PRODUCTS
    res = {"d_build_sec": wall + t_gather,
           "d_build": {"kind": "per-sample Jacobian Gram G = J J' (n x n, fp32-accurate fp16 h3 split MFMA, "
                               "fp32 sums over chunks of 5,120 k added in fp64)" +
                               (f", {world} shards of the lower-triangle tiles + RCCL "
                                f"send/recv gather to rank 0" if world > 1 else ""),
                       "n_samples": n, "n_params": model.P, "conv_columns": Kc, "ranks": world,
                       "shard_sec_max_over_ranks": wall, "gather_sec": t_gather,
                       **({"gather_check": gather_check} if gather_check else {}),
                       "phase_ms": {"forward_and_data_grads": ms[0], "per_sample_conv_jacobians": ms[1],
                                    "conv_gram": ms[2], "dense_terms_chunk_sum_and_mirror": ms[3]},
                       "naive_flop": 2.0 * n * n * model.P, "executed_gram_flop_this_rank": flop_gram,
                       "roofline": {"bound": "mfma",
                                    "kernel": "h3_rows_kernel + syrk_h3k_kernel (256 x 256 tiles, the k "
                                              "reduction split into fp32 chunks of 5,120; fp16 h3 split on "
                                              "v_mfma_f32_16x16x32_f16, LDS-DMA staged), conv-column Gram; the "
                                              "chunk sum (syrk_ksum_kernel, fp64) is in the next phase",
                                    "achieved": tf, "peak": speak, "unit": "TFLOP/s (fp32-equivalent)",
                                    "frac": tf / speak, "avg_launch_ms": ms[2], "flop_per_launch": flop_gram,
                                    "traffic": None, "half_mfma_tflops_executed": tf * H3_PRODUCTS,
                                    "mfma_utilization": tf * H3_PRODUCTS / PEAK_BF16_TFLOPS,
                                    "fp32_mfma_peak": PEAK_FP32_TFLOPS}}}
    if n == 50000 and world == 1:
        res["d_build"]["roofline"].update(_latest_pmc("syrk_h3k_kernel", "*_pmc_syrk.json"))
    tr_file = _latest_traffic("syrk_h3k_kernel", "*_syrk_traffic.json") if n == 50000 and world == 1 else None
    if tr_file:
        rf = res["d_build"]["roofline"]
        rf["traffic"] = tr_file["bytes_per_launch"]
        rf["traffic_source"] = tr_file["source"]
        rf["traffic_note"] = ("L2-miss bytes (HBM + Infinity Cache) of the Gram launch; its unique operand bytes "
                              "are the n x Kc fp16 h/l row planes (4 B per entry) + the fp32 partial tiles it "
                              "writes (one 256 x 256 tile per lower-triangle tile and chunk)")
        nch = -(-((Kc + 31) // 32) // 160)
        t256 = -(-n // 256)
        uniq = 4.0 * n * ((Kc + 31) // 32 * 32) + 4.0 * nch * (t256 * (t256 + 1) // 2) * 256 * 256
        rf["unique_operand_bytes"] = uniq
        rf["traffic_over_unique"] = rf["traffic"] / uniq
    del G, rb
    return res


def d_build(args, snk, tr) -> dict:
    """The two Laplace D builds, after the timed region, on rank 0.

    d_build_sec: G = J J' over the replay buffer's 50k per-sample Jacobians
    (north_star / configs[4]); phases timed with HIP events on the library
    stream. snapshot_gram: compute_D.jl's own D (K q_net snapshots, one per
    trainer iteration here), Welford + centring + D'D."""
    import time

    import numpy as np
    from snake_amd import _lib

    res = d_build_gram(args, snk, tr.model, None, 0, 1)
    P = tr.model.P
    K = args.d_snapshots
    if K > 1:
        lap = snk.LaplaceD(P, K)
        for pos in range(K):
            lap.snapshot(tr.model, pos)
            tr.run(1, learn=True, graph=not args.no_graph)
        _lib.call("snk_synchronize")
        t0 = time.perf_counter()
        lap.fit_center()
        _lib.call("snk_synchronize")
        t_fit = time.perf_counter() - t0
        lap.gram()                                       # first call: allocates the partial tiles
        t0 = time.perf_counter()
        _, gms = lap.gram()
        t_gram = time.perf_counter() - t0
        fl = float(K) * (K + 1) * ((P + 3) // 4 * 4)
        # la_utils.jl:97-118 at the reference's scale: K = 58 snapshots, 5000 sampled models,
        # every model one greedy episode (lockstep, per-env weights)
        lap58 = snk.LaplaceD(P, 58)
        for pos in range(58):
            tr.run(1, learn=True, graph=not args.no_graph)
            lap58.snapshot(tr.model, pos)
        lap58.fit_center()
        ls = snk.laplace_sampling_(tr, lap58, n_models=64, seed=1)          # warm-up
        _lib.call("snk_synchronize")
        t0 = time.perf_counter()
        ls = snk.laplace_sampling_(tr, lap58, n_models=5000, seed=2)
        t_ls = time.perf_counter() - t0
        msteps = int(ls["lengths"].sum())
        wbytes = 4.0 * ((P + 3) // 4 * 4)
        res["laplace_sampling"] = {"kind": "laplace_sampling! (la_utils.jl:97-118): sample_model x 5000 (K = 58) + "
                                           "one greedy episode each, lockstep on the device",
                                   "n_models": 5000, "K": 58, "seconds": t_ls, "models_per_s": 5000 / t_ls,
                                   "model_steps": msteps, "model_steps_per_s": msteps / t_ls,
                                   "mean_episode_length": float(ls["lengths"].mean()),
                                   "n_better_models": ls["n_better_models"],
                                   "weight_stream_GBs": msteps * wbytes / t_ls / 1e9,
                                   "weight_stream_frac_hbm": msteps * wbytes / t_ls / 1e9 / PEAK_HBM_GBS}
        del lap58
        ks = snk.get_arith("syrk_ksplit")
        res["snapshot_gram"] = {"kind": "compute_D.jl D (P x K Float64 snapshots) -> Welford, centre, G = D'D",
                                "K": K, "n_params": P, "welford_center_ms": 1e3 * t_fit,
                                # Welford reads D; the centring reads and writes D and writes the fp32
                                # copy (and, k-split, its fp16 h / l planes)
                                "welford_center_GBs": (32.0 if ks else 28.0) * K * P / t_fit / 1e9,
                                "gram_kernel": ("syrk_h3k_kernel: fp16 h3 split (one exponent per row and "
                                                "1024-column chunk) on v_mfma_f32_16x16x32_f16, 256 x 256 tiles, "
                                                "fp32 chunk partials summed in fp64 by syrk_ksum_kernel (in "
                                                "gram_total_ms, not in gram_kernel_ms)" if ks else
                                                "syrk_slab_kernel: bf16 x6 split, fp64 slabs"),
                                "gram_kernel_ms": gms, "gram_total_ms": 1e3 * t_gram,
                                "gram_tflops": fl / (gms * 1e-3) / 1e12,
                                "gram_frac_peak": fl / (gms * 1e-3) / 1e12 / (PEAK_BF16_TFLOPS / (H3_PRODUCTS if ks
                                                                                                   else X6_PRODUCTS))}
    return res


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # host-side barrier / max-reduce; device traffic is RCCL in-library

    import numpy as np
    import snake_amd as snk
    from snake_amd import _lib
    lib = snk.load()
    _lib.call("snk_set_device", local)
    arith_set = {}
    for kv in args.arith:
        k, v = kv.split("=")
        snk.set_arith(k, bool(int(v)))
        arith_set[k] = int(v)

    n, bs, C = args.n_envs, args.board_size, args.n_frames
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=args.capacity, batch_size=64,
                     epsilon=args.epsilon, epsilon_end=args.epsilon, decay=0.0,
                     updates_per_iter=args.updates_per_iter, seed=1234 + rank, graph_unroll=args.graph_unroll)
    comm = None
    if world > 1:
        with _stdout_to_stderr():
            comm = snk.dist_attach(tr, dist, rank, world)
    graph = not args.no_graph
    snk.fill_buffer_(tr, graph=graph)                    # fill_buffer!: untimed
    tr.run(args.warmup, learn=True, graph=graph)
    # untimed settle: the driver's windows fell monotonically after 5 warm-up steps (the
    # device's clocks still ramping), so keep iterating for args.settle_ms before timing
    _lib.call("snk_synchronize")
    t_settle, settle_iters = time.perf_counter(), 0
    while time.perf_counter() - t_settle < args.settle_ms / 1e3:
        tr.run(8, learn=True, graph=graph)
        _lib.call("snk_synchronize")
        settle_iters += 8

    def barrier():
        _lib.call("snk_synchronize")
        if dist is not None:
            dist.barrier()

    windows = []
    for _ in range(max(1, args.repeats)):
        barrier()
        t0 = time.perf_counter()
        tr.run(args.steps, learn=True, graph=graph)
        barrier()
        w = time.perf_counter() - t0
        if dist is not None:
            import torch
            t = torch.tensor([w], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            w = float(t.item())
        windows.append(w)
    elapsed = float(np.median(windows))   # median of the timed windows
    st = tr.stats()
    faults = tr.game.check_faults()
    # RCCL's own count of the group (ncclCommCount on the trainer's communicator; a one-rank
    # communicator at --gpus 1): a scaling run proves the ranks its gradient all-reduce spanned
    if comm is not None:
        rccl_nranks, rccl_rank = comm.info()
    else:
        with _stdout_to_stderr():
            c1 = snk.Comm(1, 0, snk.Comm.unique_id())
        rccl_nranks, rccl_rank = c1.info()
        del c1
    if rccl_nranks != world or rccl_rank != rank:
        print(json.dumps({"error": f"RCCL reports {rccl_nranks} ranks (this is rank {rccl_rank}); "
                                   f"WORLD_SIZE {world}, RANK {rank}"}), flush=True)
        sys.exit(3)
    if comm is not None:
        # every rank leaves the RCCL group together: rank 0's extras below keep
        # training locally (snapshots) and must not wait on ranks that have exited
        _lib.call("snk_synchronize")
        dist.barrier()
        snk.dist_detach(tr)

    out = {
        "metric": "env-steps/sec/GPU @4096 envs + D(50k) build sec, 1/2/4/8 MI355X",
        "value": world * n * args.steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "windows_ms": [1000.0 * w for w in windows],
        "windows_spread": (max(windows) - min(windows)) / elapsed,
        "settle": {"iterations": settle_iters, "ms": args.settle_ms,
                   "note": "untimed trainer iterations after the warm-up, before the timed windows"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (real Snake dynamics from SnakeGame(); glorot-initialised Q-net)",
        "config": {"workload": (f"configs[3]: {world * n} envs over {world} GPU(s), " if args.workload == "configs3"
                                else "configs[1]: ") +
                               f"{n} lockstep {bs}x{bs} envs/GPU, {C}-frame 3-action DQN: "
                               f"eps-greedy Q forward + step!/virtual_step + store! + "
                               f"{args.updates_per_iter} B=64 update(s) per step",
                   "effective_global_batch": 64 * world,
                   "batch_semantics": "B = 64 per rank per update, gradients mean-all-reduced over the ranks "
                                      "(RCCL): an effective batch of 64 x n_gpus per update"
                                      if world > 1 else "B = 64 per update",
                   "n_envs_per_gpu": n, "board_size": bs, "n_frames": C, "replay_capacity": args.capacity,
                   "batch_size": 64, "epsilon": args.epsilon, "parallelism": f"dp{world}" if world > 1 else "none",
                   "hipgraph": graph,
                   "gemm_arithmetic": ("act-forward conv2 + conv3: f32 operands as fp16 hi/lo parts of power-of-two-scaled "
                                       "values, 3 f16 MFMA products; other GEMMs: 3-way bf16 split, 6 bf16 MFMA "
                                       "products; f32 accumulation throughout"),
                   **({"arith_ab": arith_set} if arith_set else {})},
        "train_stats": {"updates": st["updates"], "episodes": st["episodes"], "env_steps": st["env_steps"],
                        "food_faults": faults},
        "rccl_nranks": rccl_nranks,
        "build": _lib.build_provenance(),
        "roofline": None,
        "cpu_baseline": None,
    }

    if rank == 0 and not args.no_extras:
        # dominant kernel: conv3 of the act forward (implicit GEMM on f32 MFMA)
        ms = np.zeros(5, np.float64)
        _lib.call("snk_dqn_time_act_layers", tr.model.handle, tr.game.handle, 20, _lib.ptr(ms))
        wo = bs - 5
        flop_conv1 = 2.0 * n * bs * bs * 16 * 9 * C
        flop_conv3 = 2.0 * n * wo * wo * (36 * 32) * 64
        flop_conv2 = 2.0 * n * bs * bs * 144 * 32
        flop_total = act_forward_flop(n, bs, C) + 2.0 * n * (wo * wo * 64 * 64 + 64 * 3)
        # ms[1] == 0: conv1 + conv2 run inside conv3's kernel (conv_h3f_kernel), ms[2] times all
        # three; ms[0] is then the conv3 weight-max scan (the h3 weight scale)
        fused = ms[1] == 0.0
        flop_dom = flop_conv3 + (flop_conv2 + flop_conv1 if fused else 0.0)
        # the dominant kernel's duration INSIDE the training loop: 50 eager training iterations,
        # each queued behind a replay of the learning graph (the GPU as busy as in the timed
        # loop), HIP events recorded by the kernel's own dispatch (hipExtLaunchKernelGGL) on the
        # library stream, the median; back to back in isolation (ms[2]) it runs slower
        loop_ms = _lib.f64(0)
        _lib.call("snk_trainer_time_act_kernel", tr.handle, 50, ctypes.byref(loop_ms))
        dom_ms = loop_ms.value if loop_ms.value > 0 else ms[2]
        tf = flop_dom / (dom_ms * 1e-3) / 1e12
        # the forward GEMMs run fp32 products as 6 exact bf16 split products on the
        # bf16 MFMA (snk.arith(conv_fp32=True): native f32 MFMA): the fp32-equivalent peak is
        # the bf16 dense peak / 6
        x6 = not snk.get_arith("conv_fp32")
        # >= 1024 samples at bs 8..13: conv_h3s_kernel (3 fp16 products per fp32 product)
        h3 = x6 and snk.get_arith("h3s") and n >= 1024 and 8 <= bs <= 13
        nprod = H3_PRODUCTS if h3 else X6_PRODUCTS
        peak = PEAK_BF16_TFLOPS / nprod if x6 else PEAK_FP32_TFLOPS
        kname = ("conv_h3f_kernel: conv1 (fp32 VALU) + conv2 + conv3 (fp16 h3 split on v_mfma_f32_16x16x32_f16) "
                 "in one kernel" if h3 and fused else
                 "conv_h3s_kernel: fp16 h3 split on v_mfma_f32_16x16x32_f16" if h3 else
                 "bf16x6 split on v_mfma_f32_16x16x32_bf16" if x6 else "v_mfma_f32_32x32x2_f32")
        out["roofline"] = {"bound": "mfma",
                           "kernel": ("conv1 + conv2 + conv3" if fused else "conv3 implicit GEMM") +
                                     ", act forward (" + kname + ")",
                           "achieved": tf, "peak": peak, "unit": "TFLOP/s (fp32-equivalent)", "frac": tf / peak,
                           "traffic": None, "avg_launch_ms": dom_ms,
                           "avg_launch_ms_how": ("median of HIP events recorded by the launch's dispatch "
                                                 "(hipExtLaunchKernelGGL) in 50 eager training iterations, each "
                                                 "queued behind a learning-graph replay"
                                                 if loop_ms.value > 0 else "HIP events, back-to-back launches"),
                           "isolated_back_to_back_ms": ms[2], "flop_per_launch": flop_dom,
                           "flop_note": "conv1's 2*n*bs^2*16*9C FLOP (1 % of the launch) run on the VALU and are "
                                        "counted against the MFMA peak" if fused else None,
                           "half_mfma_tflops_executed": tf * nprod if x6 else None,
                           "fp32_mfma_peak": PEAK_FP32_TFLOPS}
        if fused and n == 4096 and bs == 12:
            out["roofline"].update(_latest_pmc(f"conv_h3f_kernel<{bs}, 8, {C}>", "*_pmc_h3f.json"))
        tr_file = _latest_traffic(f"conv_h3f_kernel<{bs}, 8, {C}>" if fused else "conv_h3s_kernel" if h3 else "conv_x6")
        if tr_file:
            out["roofline"]["traffic"] = tr_file["bytes_per_launch"]
            out["roofline"]["traffic_source"] = tr_file["source"]
        out["act_forward_ms"] = {("wmax_scan" if fused else "conv1"): ms[0], "conv2": ms[1],
                                 ("conv1+conv2+conv3" if fused else "conv3"): ms[2],
                                 "dense1": ms[3], "head": ms[4],
                                 "total": float(ms.sum()),
                                 "tflops_total": flop_total / (ms.sum() * 1e-3) / 1e12}
        # the fused env step + store kernel (HBM roofline)
        act = snk.DeviceArray(n, np.uint8)
        snk.synth_actions_dev(tr.game, 99, act)
        sms = _lib.f64(0)
        _lib.call("snk_env_time_step", tr.game.handle, tr.buffer.handle, act.ptr, 50, ctypes.byref(sms))
        step_bytes = (C + 4) * bs * bs + 57
        gbs = n * step_bytes / (sms.value * 1e-3) / 1e9
        out["step_kernel"] = {"avg_launch_ms": sms.value, "bytes_per_env_step": step_bytes,
                              "achieved_GBs": gbs, "frac_hbm": gbs / PEAK_HBM_GBS,
                              "env_steps_per_s": n / (sms.value * 1e-3)}
        # configs[2]-scale step kernel (20x20 boards): 65,536 envs (working set inside the 256 MB
        # Infinity Cache) and 262,144 envs (HBM-resident), pure step and with the replay store fused
        out["step_kernel_large"] = []
        for ln, store in ((65536, True), (262144, False), (262144, True)):
            try:
                out["step_kernel_large"].append(step_kernel_point(snk, ln, 20, C, store))
            except Exception as e:   # report, do not fail the headline line
                out["step_kernel_large"].append({"n_envs": ln, "store": store, "error": str(e)})
    if rank == 0 and world == 1 and not args.no_extras:
        eps_rate = st["episodes"] / max(1, st["env_steps"])
        try:
            out["reference_ratio"] = reference_ratio(args, snk, graph, eps_rate)
            rr = out["reference_ratio"]
            rr["ms_per_update_marginal"] = (rr["ms_per_step"] - out["ms_per_step"]) / (rr["updates_per_step"] - 1)
            ufl = update_flop(64, bs, C)
            utf = ufl / (rr["ms_per_update_marginal"] * 1e-3) / 1e12 if rr["ms_per_update_marginal"] > 0 else 0.0
            x6peak = PEAK_BF16_TFLOPS / X6_PRODUCTS
            rr["update_roofline"] = {"bound": "mfma", "flop_per_update": ufl, "achieved": utf,
                                     "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s (fp32)",
                                     "frac": utf / PEAK_FP32_TFLOPS,
                                     "peak_x6_equivalent": x6peak, "frac_vs_x6_equivalent": utf / x6peak,
                                     "peak_note": "the update's GEMMs run on three arithmetics: the bf16 x6 split "
                                                  "(upd_fwd's conv2 / conv3, 419 TFLOP/s fp32-equivalent), the fp16 "
                                                  "h3 split (conv3_bwd / conv2_bwd data gradients, 839) and exact "
                                                  "f32 / f64 MFMA (weight gradients, Dense1, 157.3 / 78.6): frac is "
                                                  "quoted against the fp32 peak, frac_vs_x6_equivalent against the "
                                                  "peak of the arithmetic that carries most of its FLOP",
                                     "note": "4 B F (B = 64, F = the 3136->64 reference net's forward FLOP) over "
                                             "the marginal update time; the update is a chain of 5 dependent "
                                             "launches (upd_fwd with Dense1 and both heads, d1_bwd, conv3_bwd, "
                                             "conv2_bwd, grad_update), latency-bound at B = 64"}
            up = _update_pmc()
            if up:
                rr["update_roofline"]["kernels_pmc"] = up
        except Exception as e:   # report, do not fail the headline line
            out["reference_ratio"] = {"error": str(e)}
        out["updates_per_s"] = args.updates_per_iter * args.steps / elapsed
    if rank == 0 and world == 1 and not args.no_configs3 and args.workload == "configs1":
        try:
            out["configs3_per_rank"] = configs3_per_rank(args, snk, graph)
        except Exception as e:
            out["configs3_per_rank"] = {"error": str(e)}
    if rank == 0 and world == 1 and not args.no_configs2:
        try:
            out["configs2"] = configs2(args, snk, graph)
        except Exception as e:
            out["configs2"] = {"error": str(e)}
    if not args.no_dbuild:
        if world == 1:      # D(50k) + compute_D's snapshot Gram + laplace_sampling! (configs[4])
            if rank == 0:
                out.update(d_build(args, snk, tr))
        else:               # D(50k) across the ranks
            r = d_build_gram(args, snk, tr.model, dist, rank, world)
            if rank == 0:
                out.update(r)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
