"""GPU parity of the Q-net forward / DQN update against the oracle.

Tolerances (fp32 device arithmetic vs the fp64 oracle; north_star asks 1e-5
relative for fp32 Q-values):
  Q-values      |q - q_ref| <= 1e-5 * max(1, |q_ref|)
  loss          relative 1e-5
  gradients     ||g - g_ref|| <= 1e-5 * ||g_ref||  and per element
                |g - g_ref| <= 1e-5 * max|g_ref| + 1e-4 * |g_ref|
RMSProp given an identical gradient is bit-exact (same Float32 op order).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _qclose(q, qref):
    return np.all(np.abs(q - qref) <= 1e-5 * np.maximum(1.0, np.abs(qref)))


def test_params_roundtrip_flux_order(snk, golden):
    m = snk.DQNModel(10, 3, n_frames=1)
    p = golden["vanilla_params"]
    assert m.P == p.size
    m.set_params(p)
    assert np.array_equal(m.get_params(), p)
    m.set_params(p, snk.SNK_NET_TARGET)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), p)


def test_vanilla_bson_greedy_kat_on_device(snk, golden):
    """BSON vanilla weights: 129/129 greedy actions of the vanilla GIF, and
    Q-values within 1e-5 of the fp64 oracle."""
    m = snk.DQNModel(10, 3, n_frames=1)
    m.set_params(golden["vanilla_params"])
    fx = golden["vanilla1"]
    x = fx["boards_cells"][:129].astype(np.float32)[:, None, :]
    q = m(x)
    assert (q.argmax(1) == fx["act_idx"]).all()
    assert _qclose(q, golden["vanilla_q"]), np.abs(q - golden["vanilla_q"]).max()


@pytest.mark.parametrize("bs,C,B", [(12, 2, 300), (10, 2, 77), (20, 2, 40), (12, 1, 64)])
def test_forward_random_vs_oracle(snk, bs, C, B):
    rng = np.random.default_rng(bs * 10 + C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=7)
    p = m.get_params()
    assert p.size == snk.nparams(bs, C) == oracle.qnet_nparams(bs, C)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    q = m(x)
    qref = oracle.qnet_forward(bs, C, p, x)
    assert _qclose(q, qref), np.abs(q - qref).max()


def test_forward_env_and_act(snk):
    bs, C, n = 12, 2, 513
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=3)
    act = snk.DeviceArray(n, np.uint8)
    for t in range(5):
        snk.synth_actions_dev(g, 11, act)
        snk.step_indices_dev(g, act.ptr)
    q_env = m.q_env(g)
    q_ref = m(snk.assemble_state_(g))
    assert np.array_equal(q_env, q_ref)
    a0 = snk.epsilon_greedy(g, m, 0.0)
    assert np.array_equal(a0, q_env.argmax(1))
    a1 = snk.epsilon_greedy(g, m, 1.0, seed=5)
    counts = np.bincount(a1, minlength=3)
    assert counts.min() > n / 3 * 0.7


def _random_replay(snk, bs, C, n=96, T=30, seed=3):
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * T, board_size=bs, n_frames=C, batch_size=64)
    act = snk.DeviceArray(n, np.uint8)
    for t in range(T):
        snk.synth_actions_dev(g, seed, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    return g, rb


@pytest.mark.parametrize("bs,C", [(12, 2), (10, 1), (16, 2), (13, 1)])
def test_loss_and_grad_vs_oracle(snk, bs, C):
    """One DQN loss + gradient (utils.jl:442-466) on a replay batch: the fused update
    forward (upd_fwd_kernel, instantiated for board sides 8/10/12/13/16) and the
    backward. Loss within 1e-5 relative, gradient normwise 1e-5 plus an elementwise
    bound; the stack_exp float-tensor path is bit-identical to the slot path."""
    g, rb = _random_replay(snk, bs, C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=21)
    rng = np.random.default_rng(0)
    # a target net different from the online net
    tp = m.get_params() + rng.standard_normal(m.P).astype(np.float32) * 0.01
    m.set_params(tp, snk.SNK_NET_TARGET)
    idx, B = snk.sample(rb, seed=4)
    ids = idx.numpy()[:B]
    loss = m.loss_grad(rb, idx, B)
    grad = m.grad
    b = snk.stack_exp(rb, ids)
    lref, gref, _ = oracle.dqn_loss_grad(bs, C, m.get_params(), tp, b["states"], b["actions"] - 1, b["rewards"],
                                         b["next_states"], b["dones"].astype(np.uint8),
                                         b["suicidal_mask"].astype(np.uint8))
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    assert np.linalg.norm(grad - gref) <= 1e-5 * np.linalg.norm(gref)
    assert np.all(np.abs(grad - gref) <= 1e-5 * np.abs(gref).max() + 1e-4 * np.abs(gref))
    # the stack_exp-tensor path gives the identical result
    loss2 = m.loss_grad_batch(b)
    assert loss2 == loss and np.array_equal(m.grad, grad)


@pytest.mark.parametrize("bs,B", [(12, 37), (13, 64), (8, 5), (12, 1), (10, 1), (12, 3)])
def test_conv3_backward_odd_batches_vs_oracle(snk, bs, B):
    """conv3_bwd_kernel (snk_bwd3.hpp): two-sample weight-gradient chunks (an odd
    batch leaves a one-sample chunk), the data gradient's dense GEMM + col2im,
    at the smallest and largest boards it takes (Wo 3 and 8) and between.
    B = 1: conv2's gradient plan has a single slab (written straight into grad,
    no K-split), which grad_update_kernel's two-thread conv2 finish once counted
    twice (a doubled conv2 gradient and RMSProp step at B = 1)."""
    g, rb = _random_replay(snk, bs, 2, n=48, T=6, seed=bs)
    m = snk.DQNModel(bs, 3, n_frames=2, seed=bs + 3)
    rng = np.random.default_rng(B)
    tp = m.get_params() + rng.standard_normal(m.P).astype(np.float32) * 0.01
    m.set_params(tp, snk.SNK_NET_TARGET)
    ids = rng.choice(48 * 6, size=B, replace=False)
    b = snk.stack_exp(rb, ids)
    loss = m.loss_grad_batch(b)
    grad = m.grad
    lref, gref, _ = oracle.dqn_loss_grad(bs, 2, m.get_params(), tp, b["states"], b["actions"] - 1, b["rewards"],
                                         b["next_states"], b["dones"].astype(np.uint8),
                                         b["suicidal_mask"].astype(np.uint8))
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    assert np.linalg.norm(grad - gref) <= 1e-5 * np.linalg.norm(gref)
    assert np.all(np.abs(grad - gref) <= 1e-5 * np.abs(gref).max() + 1e-4 * np.abs(gref))


@pytest.mark.parametrize("scale", [1e2, 1e4])
def test_backward_wide_dynamic_range_vs_oracle(snk, scale):
    """The conv3 / conv2 data gradients run on the fp16 h3 split with ONE power-of-two
    scale per sample (dz) and per block (weights): an element far below its sample's
    maximum keeps only what the fp16 subnormal range holds of its low part (absolute
    error <= 2^-40 of the scaled maximum, DESIGN.md §4 "Error bound of the h3 data gradients"). Here a few Dense1
    weight columns are scaled by `scale`, so dz3 of each sample has a handful of
    entries `scale` times larger than the rest and dz2 inherits the spread. Every
    parameter section's gradient (conv1, conv2, conv3, Dense1 weights) must still
    match the fp64 oracle normwise within 1e-5 of that section's own norm, so a
    precision loss in the small entries cannot hide behind the large ones."""
    bs, C = 12, 2
    g, rb = _random_replay(snk, bs, C, seed=11)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=31)
    rng = np.random.default_rng(int(scale))
    p = m.get_params()
    sec = [9 * C * 16, 16, 144 * 32, 32, 1152 * 64, 64, 3136 * 64, 64, 192, 3]
    off = np.concatenate([[0], np.cumsum(sec)])
    d1 = p[off[6]:off[7]].reshape(3136, 64)          # Flux W (64, 3136) column-major: [f][o]
    cols = rng.choice(3136, 4, replace=False)
    d1[cols] *= np.float32(scale)
    p[off[6]:off[7]] = d1.reshape(-1)
    m.set_params(p)
    tp = p + rng.standard_normal(m.P).astype(np.float32) * 0.01
    m.set_params(tp, snk.SNK_NET_TARGET)
    idx, B = snk.sample(rb, seed=5)
    loss = m.loss_grad(rb, idx, B)
    grad = m.grad
    b = snk.stack_exp(rb, idx.numpy()[:B])
    lref, gref, _ = oracle.dqn_loss_grad(bs, C, p, tp, b["states"], b["actions"] - 1, b["rewards"], b["next_states"],
                                         b["dones"].astype(np.uint8), b["suicidal_mask"].astype(np.uint8))
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    for k, name in ((0, "conv1 W"), (2, "conv2 W"), (4, "conv3 W"), (6, "Dense1 W")):
        gs, rs = grad[off[k]:off[k + 1]], gref[off[k]:off[k + 1]]
        e = np.linalg.norm(gs - rs) / np.linalg.norm(rs)
        print(f"scale {scale:g} {name}: normwise {e:.2e}")
        assert e <= 1e-5, (name, e)


def test_rmsprop_bitexact(snk):
    m = snk.DQNModel(12, 3, n_frames=2, seed=5)
    rng = np.random.default_rng(1)
    P = m.P
    g = (rng.standard_normal(P) * 10.0 ** rng.uniform(-9, 0, P)).astype(np.float32)
    acc = (np.abs(rng.standard_normal(P)) * 1e-3).astype(np.float32)
    acc[::7] = 0
    th = m.get_params()
    m.set_params(g, snk.SNK_NET_GRAD)
    m.set_params(acc, snk.SNK_NET_OPT_STATE)
    for _ in range(3):
        m.apply_grad()
        th, acc = oracle.rmsprop(th, acc, g)
    assert np.array_equal(m.get_params(), th)
    assert np.array_equal(m.get_params(snk.SNK_NET_OPT_STATE), acc)


def test_update_and_target_sync(snk):
    g, rb = _random_replay(snk, 12, 2)
    m = snk.DQNModel(12, 3, n_frames=2, seed=8)
    th0 = m.get_params()
    idx, B = snk.sample(rb, seed=9)
    loss = m.loss_grad(rb, idx, B)
    grad = m.grad
    m.apply_grad()
    th1, _ = oracle.rmsprop(th0, np.zeros_like(th0), grad)
    assert np.array_equal(m.get_params(), th1)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), th0)
    snk.update_target_net_(m)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), th1)
    assert np.isfinite(loss)


def test_trainer_schedule_and_graph_determinism(snk):
    """train!: fill the buffer, n_batches+1 updates, epsilon decay per update
    (Float32, utils.jl:480), target sync at nb % rate == 0; the captured
    hipGraph replay is bit-identical to eager launches."""
    outs = []
    for graph in (False, True):
        tr = snk.Trainer(n_batches=40, target_update_rate=16, n_envs=128, board_size=12, n_frames=2,
                         capacity=1000, decay=1e-3, seed=77)
        st = snk.train_(tr, graph=graph)
        outs.append((tr.model.get_params(), tr.model.get_params(snk.SNK_NET_TARGET), tr.losses, st))
    (p0, t0, l0, s0), (p1, t1, l1, s1) = outs
    assert np.array_equal(p0, p1) and np.array_equal(t0, t1) and np.array_equal(l0, l1)
    assert s0["updates"] == 41 and s1 == s0
    eps = np.float32(1.0)
    for _ in range(41):
        eps = max(np.float32(eps - np.float32(1e-3)), np.float32(0.05))
    assert np.float32(s0["epsilon"]) == eps
    assert len(l0) == 41 and np.all(np.isfinite(l0))
    assert s0["env_steps"] >= 1001 and s0["episodes"] > 0


def test_trainer_alternating_tail_graphs_match_eager(snk):
    """run() lengths that leave alternating remainders (graph_unroll 4: 3, 5 -> 4 + 1,
    3, 2, 6 -> 4 + 2, 3, 1) replay cached tail graphs (the 3 most recently used per learn mode)
    and capture new ones as they come; every iteration equals the eager launch sequence bit for
    bit (both nets, losses, counters)."""
    outs = []
    for graph in (False, True):
        tr = snk.Trainer(n_envs=128, board_size=12, n_frames=2, capacity=2000, batch_size=64, n_batches=10_000,
                         target_update_rate=5, decay=1e-3, seed=78, graph_unroll=4)
        snk.fill_buffer_(tr, graph=graph)
        for it in (3, 5, 3, 2, 6, 3, 1, 2, 3):
            tr.run(it, learn=True, graph=graph)
        outs.append((tr.model.get_params(), tr.model.get_params(snk.SNK_NET_TARGET), np.array(tr.losses)))
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
    assert outs[0][2].size == 28 and np.isfinite(outs[0][2]).all()


@pytest.mark.parametrize("bs,C,B", [(12, 2, 300), (10, 1, 257)])
def test_x6_split_forward_matches_fp32_and_oracle(snk, bs, C, B):
    """The bf16x6 split-precision forward (default) has the error class of the
    exact-fp32 MFMA forward (snk.arith(conv_fp32=True)): at the init scale both meet the
    1e-5 bar against the fp64 oracle; with 3x larger weights (|Q| ~ 100 with
    heavy cancellation, where fp32 itself exceeds 1e-5) the x6 error stays
    within 2x the fp32 error, element-max and mean."""
    rng = np.random.default_rng(bs * 100 + B)
    m6 = snk.DQNModel(bs, 3, n_frames=C, seed=5)
    with snk.arith(conv_fp32=True):
        m32 = snk.DQNModel(bs, 3, n_frames=C, seed=5)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    p0 = m6.get_params()
    for scale in (1.0, 3.0):
        p = p0 * np.float32(scale)
        m6.set_params(p)
        m32.set_params(p)
        q6, q32 = m6.forward(x), m32.forward(x)
        qref = oracle.qnet_forward(bs, C, p, x)
        e6 = np.abs(q6 - qref) / np.maximum(1.0, np.abs(qref))
        e32 = np.abs(q32 - qref) / np.maximum(1.0, np.abs(qref))
        if scale == 1.0:
            assert e6.max() <= 1e-5 and e32.max() <= 1e-5
        assert e6.max() <= 2 * e32.max() + 1e-7, (scale, e6.max(), e32.max())
        assert e6.mean() <= 2 * e32.mean() + 1e-8, (scale, e6.mean(), e32.mean())


def test_large_batch_forward_h3s_vs_oracle(snk):
    """B >= 1024 routes conv3 through conv_h3s_kernel (fp16 h3 split, four
    samples' inputs in LDS). 1101 samples leave a partial last group of one
    sample. Tolerance: |q - q_ref| <= 1e-5 * max(1, |q_ref|)."""
    bs, C, B = 12, 2, 1101
    rng = np.random.default_rng(11)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=13)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    q = m(x)
    qref = oracle.qnet_forward(bs, C, m.get_params(), x)
    assert _qclose(q, qref), np.abs(q - qref).max()


@pytest.mark.parametrize("bs,C", [(8, 1), (10, 2), (13, 2)])
def test_large_batch_forward_h3_board_sizes(snk, bs, C):
    """conv2 (conv_h3c2_kernel, two samples per workgroup) and conv3 on the h3
    split at the other board sides: at 10 and 13 a 16-row tile straddles the
    two samples (per-row exponents), 1027 samples leave a one-sample last
    workgroup. Tolerance as the 12x12 case."""
    rng = np.random.default_rng(bs)
    B = 1027
    m = snk.DQNModel(bs, 3, n_frames=C, seed=bs + 1)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    q = m(x)
    qref = oracle.qnet_forward(bs, C, m.get_params(), x)
    assert _qclose(q, qref), np.abs(q - qref).max()


@pytest.mark.parametrize("scale", [1.0, 3.0, 1e-3, 40.0])
def test_h3s_error_class_vs_fp32(snk, scale):
    """The h3 conv3 (fp16 parts of power-of-two-scaled operands, 3 MFMAs per
    product) keeps the error class of the exact-fp32 MFMA forward
    (snk.arith(conv_fp32=True)) across weight scales that move activations over 10+
    binades (1e-3x: tiny activations, where unscaled fp16 would underflow;
    40x: |Q| ~ 1e8, where it would overflow): element-max and mean error
    against the fp64 oracle within 4x the fp32 forward's (its operands carry
    2^-22 representation error where fp32 MFMA operands are exact; measured
    ~2x), and within 1e-5 at the init scale."""
    bs, C, B = 12, 2, 1030
    rng = np.random.default_rng(7)
    mh = snk.DQNModel(bs, 3, n_frames=C, seed=5)
    with snk.arith(conv_fp32=True):
        m32 = snk.DQNModel(bs, 3, n_frames=C, seed=5)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    p = mh.get_params() * np.float32(scale)
    mh.set_params(p)
    m32.set_params(p)
    qh, q32 = mh.forward(x), m32.forward(x)
    qref = oracle.qnet_forward(bs, C, p, x)
    if scale == 1.0:
        assert _qclose(qh, qref) and _qclose(q32, qref)
    # relative error, floored at 1e-3 of the largest |Q| (scale-free)
    den = np.maximum(np.abs(qref), 1e-3 * np.abs(qref).max())
    eh = np.abs(qh - qref) / den
    e32 = np.abs(q32 - qref) / den
    print(f"h3s scale {scale}: max {eh.max():.3e} (fp32 {e32.max():.3e}), mean {eh.mean():.3e} (fp32 {e32.mean():.3e})")
    assert eh.max() <= 4 * e32.max() + 1e-7, (scale, eh.max(), e32.max())
    assert eh.mean() <= 4 * e32.mean() + 1e-8, (scale, eh.mean(), e32.mean())


def test_x6s_bitexact_with_x6m16_and_h3s_close(snk):
    """With the h3 kernel off (snk.arith(h3s=False)), conv_x6s accumulates the six
    part products in x6m16's order: the Q values of a 2050-sample forward are
    identical with x6s on and off. The default forward (conv2 and conv3 on h3)
    and the h3-conv3-only one (h3c2=False) agree with them to 1e-5 * max(1, |q|).
    The knobs are the snk_set_arith ABI call (no environment variable changes the
    shipping library's arithmetic)."""
    out = {}
    for tag, knobs in (("x6s", dict(h3s=False, x6s=True)), ("m16", dict(h3s=False, x6s=False)),
                       ("h3c3", dict(h3c2=False)), ("h3s", {})):
        rng = np.random.default_rng(4)
        m = snk.DQNModel(12, 3, n_frames=2, seed=21)
        x = rng.integers(-1, 3, size=(2050, 2, 144)).astype(np.float32)
        with snk.arith(**knobs):
            out[tag] = m(x)
    assert np.array_equal(out["x6s"], out["m16"])
    assert _qclose(out["h3s"], out["x6s"]) and _qclose(out["h3c3"], out["x6s"])
    assert not np.array_equal(out["h3s"], out["x6s"]), "snk.arith(h3s=False) did not switch the conv3 kernel"


def test_train_episode_schedule(snk):
    """train_(tr, schedule="episode") runs utils.jl:389-482 literally: fill
    until more than `capacity` transitions were played, then n_batches + 1
    rounds of (one epsilon-greedy episode stored, one B=64 update), the
    target synced when nb % rate == 0 (rate 1: after every update, so t_net
    ends equal to q_net), epsilon decayed per update in Float32 and clamped
    at epsilon_end. Deterministic for a fixed seed."""
    outs = []
    for _ in range(2):
        tr = snk.Trainer(n_envs=1, board_size=10, n_frames=2, capacity=300, n_batches=12, target_update_rate=1,
                         epsilon=1.0, epsilon_end=0.6, decay=0.05, seed=3)
        st = snk.train_(tr, schedule="episode")
        outs.append((tr.model.get_params(), tr.model.get_params(snk.SNK_NET_TARGET), list(tr.episode_losses),
                     list(tr.episode_rewards), st))
    (p0, t0, l0, r0, s0), (p1, t1, l1, r1, s1) = outs
    assert np.array_equal(p0, t0), "rate 1: t_net synced after the last update"
    assert np.array_equal(p0, p1) and l0 == l1 and r0 == r1
    assert s0["updates"] == 13 and len(l0) == 13 and len(r0) == 13
    assert np.all(np.isfinite(l0)) and all(r <= 60 for r in r0)
    eps = np.float32(1.0)
    for _ in range(13):
        eps = max(np.float32(eps - np.float32(0.05)), np.float32(0.6))
    assert np.float32(s0["epsilon"]) == eps
    assert s0["buffer_length"] == 300


@pytest.mark.parametrize("n_envs", [4096, 200])
def test_trainer_episode_stats_fold(snk, n_envs):
    """The step kernel's last workgroup folds the finished episodes into the
    trainer statistics (episode_stats, utils.jl:478) and advances the step and
    replay counters. Checked iteration by iteration against the step's own
    outputs accumulated on the host: episodes, score sum, reward max, score max
    and env-steps exact; the Float64 reward sum within 1e-12 relative (the
    device reduces per-workgroup partials in workgroup order). 200 envs leave a
    partial last workgroup."""
    tr = snk.Trainer(n_batches=10, n_envs=n_envs, board_size=12, n_frames=2, capacity=4 * n_envs, epsilon=1.0,
                     decay=0.0, seed=3)
    s0 = tr.stats()
    t0 = tr.game.t
    ep, ss, rs, rm, sm = 0, 0, 0.0, -np.inf, 0
    for it in range(60):
        tr.run(1, learn=False, graph=(it % 2 == 0))
        o = tr.game.last("done", "ep_reward", "score")
        d = o["done"].astype(bool)
        ep += int(d.sum())
        ss += int(o["score"][d].astype(np.int64).sum())
        rs += float(o["ep_reward"][d].astype(np.float64).sum())
        if d.any():
            rm = max(rm, float(o["ep_reward"][d].max()))
            sm = max(sm, int(o["score"][d].max()))
    st = tr.stats()
    assert ep > 0
    assert st["episodes"] - s0["episodes"] == ep
    assert st["score_sum"] - s0["score_sum"] == ss
    assert st["env_steps"] - s0["env_steps"] == 60 * n_envs
    assert np.float32(st["reward_max"]) == np.float32(rm) and st["score_max"] == sm
    assert abs(st["reward_sum"] - rs) <= 1e-12 * max(1.0, abs(rs))
    assert tr.game.t == t0 + 60
    assert len(tr.buffer) == min(60 * n_envs, 4 * n_envs)


@pytest.mark.parametrize("bs,C", [(9, 2), (10, 1), (11, 2), (13, 1), (13, 2)])
def test_h3f_act_forward_boards_vs_oracle(snk, bs, C):
    """conv_h3f_kernel (conv1 on the VALU in fp32, conv2 + conv3 on the h3 split; >= 1024
    states) at the other board sides it serves: odd sides leave a partial conv1 tile per group,
    13 runs the register-staged (non-DMA) form, 1100 states a partial last group of four.
    Q of every 7th state and the last four within 1e-5 * max(1, |q|) of the fp64 oracle."""
    rng = np.random.default_rng(bs * 10 + C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=31)
    p = m.get_params()
    x = rng.integers(-1, 3, size=(1100, C, bs * bs)).astype(np.float32)
    q = m(x)
    sel = np.concatenate([np.arange(0, 1100, 7), np.arange(1096, 1100)])
    qref = oracle.qnet_forward(bs, C, p, x[sel])
    err = np.abs(q[sel] - qref) / np.maximum(1.0, np.abs(qref))
    assert err.max() <= 1e-5, float(err.max())


def test_dense_h3_act_forward(snk):
    """Dense1 of the 4096-state act forward on dense_h3_kernel (fp16 h3 split, per-sample
    a3 scale from conv_h3f's epilogue, per-(position, output) weight scales from
    w3_split_kernel) against the same forward with Dense1 on the x6 kernel
    (snk.arith(dh3=False)): 2e-6 * max(1, |q|) at most, 3e-7 on average; both against
    the fp64 oracle at 1e-5."""
    out = {}
    for flag in (True, False):
        rng = np.random.default_rng(6)
        m = snk.DQNModel(12, 3, n_frames=2, seed=23)
        x = rng.integers(-1, 3, size=(4096, 2, 144)).astype(np.float32)
        with snk.arith(dh3=flag):
            out[flag] = (m(x), m.get_params())
    qh, p = out[True]
    qx, _ = out[False]
    assert np.array_equal(p, out[False][1])
    assert not np.array_equal(qh, qx), "snk.arith(dh3=False) did not switch the Dense1 kernel"
    # measured spread of the two exact-split paths: max 3.7e-7, mean 6.9e-8 (round 4); a wrong
    # row or column scale (the round-4 a3-max bug) shows up far above these bounds
    rel = np.abs(qh - qx) / np.maximum(1.0, np.abs(qx))
    print(f"dense_h3 vs x6: max {rel.max():.3e}, mean {rel.mean():.3e}")
    assert rel.max() <= 2e-6 and rel.mean() <= 3e-7, (float(rel.max()), float(rel.mean()))
    rng = np.random.default_rng(6)
    x = rng.integers(-1, 3, size=(4096, 2, 144)).astype(np.float32)
    sel = np.arange(0, 4096, 16)
    qref = oracle.qnet_forward(12, 2, p, x[sel])
    for q in (qh, qx):
        err = np.abs(q[sel] - qref) / np.maximum(1.0, np.abs(qref))
        assert err.max() <= 1e-5, float(err.max())


@pytest.mark.parametrize("B", [64, 37])
def test_update_heads_fused_bitexact(snk, B):
    """The update's two heads (t_net TD target, q_net Huber loss / dq / dz1) in upd_fwd_kernel's
    tail (sc1 slab hand-off, per-sample ticket) against head_pair_kernel
    (snk.arith(upd_head=False)): loss and gradient bit-identical."""
    g, rb = _random_replay(snk, 12, 2)
    m = snk.DQNModel(12, 3, n_frames=2, seed=21)
    rng = np.random.default_rng(1)
    m.set_params(m.get_params() + rng.standard_normal(m.P).astype(np.float32) * 0.01, snk.SNK_NET_TARGET)
    idx, _ = snk.sample(rb, seed=4)
    res = {}
    for fused in (True, False):
        with snk.arith(upd_head=fused):
            loss = m.loss_grad(rb, idx, B)
            res[fused] = (loss, m.grad.copy())
    assert res[True][0] == res[False][0]
    assert np.array_equal(res[True][1], res[False][1])


def _handoff_case(snk, B=64):
    """One update's loss and gradient through upd_fwd_kernel's fused heads (the sc1 slab
    hand-off in the shipping build), on fixed inputs."""
    g, rb = _random_replay(snk, 12, 2)
    m = snk.DQNModel(12, 3, n_frames=2, seed=21)
    rng = np.random.default_rng(1)
    m.set_params(m.get_params() + rng.standard_normal(m.P).astype(np.float32) * 0.01, snk.SNK_NET_TARGET)
    idx, _ = snk.sample(rb, seed=4)
    loss = m.loss_grad(rb, idx, B)
    return np.float64(loss), m.grad.copy()


def test_update_sc1_handoff_matches_acq_rel_build(snk, tmp_path):
    """upd_fwd_kernel hands the Dense1 slabs to the sample's last workgroup
    with sc1 stores, an in-order vmcnt wait and a relaxed ticket: an ISA-level argument
    (snk_upd_fwd.hpp), not a C++ happens-before. The formally ordered build (-DUPD_SC1=0: an
    acq_rel ticket, libsnakehip_acqrel.so, built by __graft_entry__.build()) runs the same update
    in a child process: loss and gradient bit-identical, for B = 64 and 37."""
    import os
    import subprocess
    import sys
    from snake_amd import _lib
    lib = os.path.join(os.path.dirname(_lib.LIB_PATH), "libsnakehip_acqrel.so")
    assert os.path.exists(lib), "libsnakehip_acqrel.so is not built (__graft_entry__.build())"
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for B in (64, 37):
        out = tmp_path / f"acq{B}.npz"
        code = (f"import sys; sys.path[:0] = [{root!r}, {here!r}, {os.path.join(root, 'oracle')!r}]\n"
                "import numpy as np, snake_amd as snk\n"
                "from snake_amd import _lib\n"
                "assert _lib.LIB_PATH.endswith('libsnakehip_acqrel.so')\n"
                "from test_qnet_gpu import _handoff_case\n"
                f"loss, grad = _handoff_case(snk, {B})\n"
                f"np.savez({str(out)!r}, loss=loss, grad=grad)\n")
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SNK_LIB=lib), check=True, timeout=240)
        ref = np.load(out)
        loss, grad = _handoff_case(snk, B)
        assert loss == ref["loss"], (float(loss), float(ref["loss"]))
        assert np.array_equal(grad, ref["grad"])


def test_env_fused_act_head_bitexact(snk):
    """The trainer's act head inside env_step_kernel (4096 envs: the act forward stops at
    Dense1's slabs; the step computes each env's Q-values and epsilon-greedy action first,
    four threads per env, Dense2 in wave_sum's butterfly order) against head_kernel<HEAD_ACT>
    (snk.arith(env_head=False)): 16 captured iterations with learning after the fill, every
    iteration's actions and Q-values, the losses and both nets bit-identical."""
    n, U = 4096, 8
    res = {}
    for fused in (True, False):
        with snk.arith(env_head=fused):
            tr = snk.Trainer(n_envs=n, board_size=12, n_frames=2, capacity=20_000, batch_size=64, n_batches=10_000,
                             epsilon=0.3, epsilon_end=0.3, decay=0.0, seed=0xE4, graph_unroll=U)
            snk.fill_buffer_(tr, graph=True)
            # zero-filled rings: a captured graph's iterations reuse their slots (slot = iteration
            # within the graph), so slots past the unroll stay as allocated
            acts = snk.DeviceArray.from_host(np.zeros((2 * U, n), np.uint8))
            qs = snk.DeviceArray.from_host(np.zeros((2 * U, n, 3), np.float32))
            tr.set_act_trace(acts, qs)
            tr.run(2 * U, learn=True, graph=True)
            res[fused] = (acts.numpy(), qs.numpy(), np.array(tr.losses), tr.model.get_params(),
                          tr.model.get_params(snk.SNK_NET_TARGET))
    for x, y in zip(res[True], res[False]):
        assert np.array_equal(x, y)
    a, q = res[True][0][:U], res[True][1][:U]
    assert 0.05 < (a != q.argmax(2)).mean() < 0.3   # the epsilon draws took effect (0.3 x 2/3 at most)


def test_split_chain_matches_fresh_splits(snk):
    """The trainer's chained act forwards (grad_update writes conv2 / conv3 / Dense1's split images
    with the exponents of the graph's first w3_split_kernel; the act forward skips the split launch)
    against a w3_split_kernel launch every iteration (snk.arith(split_chain=False)): while no
    weight maximum crosses a power of two inside a graph the exponents agree and so do the bits;
    16 captured iterations with learning at 4096 envs: actions, Q-values, losses, both nets."""
    n, U = 4096, 8
    res = {}
    for chained in (True, False):
        with snk.arith(split_chain=chained):
            tr = snk.Trainer(n_envs=n, board_size=12, n_frames=2, capacity=20_000, batch_size=64, n_batches=10_000,
                             epsilon=0.05, epsilon_end=0.05, decay=0.0, seed=0x5C, graph_unroll=U)
            snk.fill_buffer_(tr, graph=True)
            acts = snk.DeviceArray.from_host(np.zeros((U, n), np.uint8))
            qs = snk.DeviceArray.from_host(np.zeros((U, n, 3), np.float32))
            tr.set_act_trace(acts, qs)
            tr.run(2 * U, learn=True, graph=True)
            res[chained] = (acts.numpy(), qs.numpy(), np.array(tr.losses), tr.model.get_params(),
                            tr.model.get_params(snk.SNK_NET_TARGET))
    for x, y in zip(res[True], res[False]):
        assert np.array_equal(x, y)


def test_split_chain_exponent_cap_keeps_q_finite(snk):
    """a chained split reuses the exponents of the graph's first w3_split_kernel, and
    RMSProp moves a weight by up to lr / sqrt(1 - rho) per step whatever its size, so a tensor (or
    Dense1 row) with a tiny maximum would grow past the fp16 range of its split within a graph.
    w3_split_kernel caps the exponents with the trainer's bound on that movement
    (snk_conv_h3f.hpp h3_exp_w). Here conv3's whole tensor and one Dense1 row start at 1e-3 of
    their glorot scale (maxima ~1e-4, 30x growth after two steps): 16 captured iterations
    with learning must keep every Q-value, loss and weight finite, and the chained run must
    match fresh splits every iteration (split_chain=False) to the h3 error class."""
    n, U = 4096, 16
    res = {}
    for chained in (True, False):
        with snk.arith(split_chain=chained):
            tr = snk.Trainer(n_envs=n, board_size=12, n_frames=2, capacity=20_000, batch_size=64, n_batches=10_000,
                             epsilon=0.05, epsilon_end=0.05, decay=0.0, seed=0x5D, graph_unroll=U)
            snk.fill_buffer_(tr, graph=True)
            th = tr.model.get_params()
            c3 = (9 * 2 * 16 + 16) + (9 * 16 * 32 + 32)        # conv3 weights (Flux order)
            d1 = c3 + 36 * 32 * 64 + 64                        # Dense1 W (64 x 3136, column-major)
            th[c3:c3 + 36 * 32 * 64] *= 1e-3
            th[d1:d1 + 64 * 3136:64] *= 1e-3                   # row (output) 0
            m_row0 = float(np.abs(th[d1:d1 + 64 * 3136:64]).max())
            tr.model.set_params(th)
            tr.model.set_params(th, snk.SNK_NET_TARGET)
            acts = snk.DeviceArray.from_host(np.zeros((U, n), np.uint8))
            qs = snk.DeviceArray.from_host(np.zeros((U, n, 3), np.float32))
            tr.set_act_trace(acts, qs)
            tr.run(U, learn=True, graph=True)
            res[chained] = (acts.numpy(), qs.numpy(), np.array(tr.losses), tr.model.get_params())
    a, q, loss, th = res[True]
    assert np.isfinite(q).all() and np.isfinite(loss).all() and np.isfinite(th).all()
    # the scenario happened: the row grew far past the 32x its split's headroom alone allows
    assert np.abs(th[d1:d1 + 64 * 3136:64]).max() > 32 * m_row0
    # the same trajectory while the actions agree (the capped exponents change only the split's
    # 2^-22 representation error)
    a2, q2, _, _ = res[False]
    for t in range(U):
        np.testing.assert_allclose(q[t], q2[t], rtol=1e-4, atol=1e-6 * np.abs(q2[t]).max())
        if not np.array_equal(a[t], a2[t]):
            break
