"""configs[2]: the deeper bf16 conv Q-net (include/snakehip.h
snk_dqn_create_deep) against the oracle's restatement of the
same bf16 arithmetic (oracle/snake_oracle.c orc_deep_*: bf16-rounded conv /
Dense1 weights and conv activations, fp64 sums).

Tolerances (bf16 storage, fp32 MFMA sums against fp64 sums: an activation
whose fp32 and fp64 values round to different bf16 neighbours moves by one
bf16 ulp, 2^-8 relative; measured values are printed):
  Q-values        |q - q_ref| <= 2e-3 * max(1, max_batch |q_ref|)
  loss            relative 2e-3
  gradient        ||g - g_ref|| <= 1e-3 * ||g_ref||   (measured ~1e-4)
  RMSProp step    bit-exact given the device gradient
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _err(q, qref):
    return float(np.max(np.abs(q - qref)) / max(1.0, float(np.abs(qref).max())))


def _close(q, qref, tol=2e-3):
    return _err(q, qref) <= tol


def _scaled(m, rng, scale=2.0):
    """glorot init gives |Q| ~ 1e-2; doubling every weight (2^6 through the
    six layers) makes Q O(1), a stricter numerical test."""
    p = m.get_params()
    p = (p * np.float32(scale)).astype(np.float32)
    m.set_params(p)
    m.set_params(p, 1)
    return p


@pytest.mark.parametrize("bs,C,B", [(10, 2, 24), (20, 2, 40), (12, 1, 17)])
def test_deep_forward_vs_oracle(snk, bs, C, B):
    m = snk.DQNModel(bs, 3, n_frames=C, seed=11, deep=True)
    assert m.P == snk.deep_nparams(bs, C) == oracle.deep_nparams(bs, C)
    rng = np.random.default_rng(bs + B)
    p = _scaled(m, rng)
    assert np.array_equal(m.get_params(), p)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    q = m.forward(x)
    qref = oracle.deep_forward(bs, C, p, x)
    err = _err(q, qref)
    print(f"deep forward bs {bs} B {B}: max err {err:.2e}, |Q| max {np.abs(qref).max():.2f}")
    assert _close(q, qref), err


def test_deep_forward_large_batch_split_paths(snk):
    """1100 samples: the L0 kernel stages several samples per workgroup and
    Dense1 runs unsplit; the sampled Q-values match the oracle and the first
    24 equal a 24-sample forward's to 1e-5 (the Dense1 K splits differ, which
    changes only the fp32 summation grouping of the head's slabs)."""
    bs, C = 20, 2
    m = snk.DQNModel(bs, 3, n_frames=C, seed=12, deep=True)
    rng = np.random.default_rng(5)
    p = _scaled(m, rng)
    x = rng.integers(-1, 3, size=(1100, C, bs * bs)).astype(np.float32)
    q = m.forward(x)
    sel = np.arange(0, 1100, 55)
    assert _close(q[sel], oracle.deep_forward(bs, C, p, x[sel]))
    q24 = m.forward(x[:24])
    assert _err(q24, q[:24]) <= 1e-5, _err(q24, q[:24])


def test_deep_forward_ragged_large_batch(snk):
    """65,636 samples: not a multiple of the 256 rows of a deep_dense1_ldsb_kernel workgroup
    (its last workgroup reads clamped a3 blocks and stores 100 rows) nor of L3's 16-sample
    a3 blocks. Sampled rows across the batch and the ragged tail match the oracle; the
    first 65,536 rows equal a 65,536-sample forward's bit for bit (every layer's per-sample
    result, Dense1's unsplit K included, is independent of the batch size)."""
    bs, C = 20, 2
    m = snk.DQNModel(bs, 3, n_frames=C, seed=12, deep=True)
    rng = np.random.default_rng(7)
    p = _scaled(m, rng)
    n = 65536 + 100
    x = rng.integers(-1, 3, size=(n, C, bs * bs)).astype(np.float32)
    q = m.forward(x)
    sel = np.r_[np.linspace(0, n - 101, 12).astype(np.int64), np.arange(n - 100, n, 9), n - 1]
    assert _close(q[sel], oracle.deep_forward(bs, C, p, x[sel]))
    q0 = m.forward(x[:65536])
    assert np.array_equal(q0, q[:65536])


def _replay(snk, bs, C, n=64, T=10, seed=3):
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * T, board_size=bs, n_frames=C, batch_size=64)
    act = snk.DeviceArray(n, np.uint8)
    for _ in range(T):
        snk.synth_actions_dev(g, seed, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    return rb


@pytest.mark.parametrize("bs,C", [(10, 2), (12, 2), (20, 2)])
def test_deep_loss_grad_and_update_vs_oracle(snk, bs, C):
    """One DQN update of the deep net on a replay batch: Huber loss and the
    bf16-MFMA gradient vs the oracle (same rounding points), RMSProp on the
    device gradient bit-exact, the new q_net's forward images consistent
    (Q after the step vs the oracle at the new parameters), t_net unchanged
    until update_target_net!."""
    rb = _replay(snk, bs, C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=21, deep=True)
    rng = np.random.default_rng(0)
    p = _scaled(m, rng)
    tp = (p + rng.standard_normal(m.P).astype(np.float32) * np.float32(0.01)).astype(np.float32)
    m.set_params(tp, snk.SNK_NET_TARGET)
    idx, B = snk.sample(rb, seed=4)
    ids = idx.numpy()[:B]
    loss = m.loss_grad(rb, idx, B)
    g = m.grad
    b = snk.stack_exp(rb, ids)
    lref, gref, _ = oracle.deep_loss_grad(bs, C, p, tp, b["states"], b["actions"] - 1, b["rewards"],
                                          b["next_states"], b["dones"].astype(np.uint8),
                                          b["suicidal_mask"].astype(np.uint8))
    gerr = np.linalg.norm(g - gref) / np.linalg.norm(gref)
    print(f"deep bs {bs}: loss {loss:.6f} vs {lref:.6f}; gradient normwise err {gerr:.2e}")
    assert abs(loss - lref) <= 2e-3 * abs(lref)
    assert gerr <= 1e-3
    # every layer's block on its own (a wrong L3 weight or bias gradient must not hide
    # inside the Dense1 block's norm): the Flux.destructure order of structs.jl:127-139
    o, blocks = 0, []
    for ks, ci, co in ((3, C, 32), (3, 32, 32), (3, 32, 64), (6, 64, 64)):
        blocks += [(f"conv{len(blocks) // 2}.w", o, o + ks * ks * ci * co)]
        o += ks * ks * ci * co
        blocks += [(f"conv{len(blocks) // 2}.b", o, o + co)]
        o += co
    K1 = (bs - 5) ** 2 * 64
    blocks += [("d1.w", o, o + K1 * 64), ("d1.b", o + K1 * 64, o + K1 * 64 + 64)]
    assert o + K1 * 64 + 64 + 3 * 64 + 3 == m.P
    for name, a, b_ in blocks:
        e = np.linalg.norm(g[a:b_] - gref[a:b_]) / max(np.linalg.norm(gref[a:b_]), 1e-30)
        print(f"  {name}: normwise err {e:.2e}")
        assert e <= 2e-3, name
    m.apply_grad()
    th1, _ = oracle.rmsprop(p, np.zeros_like(p), g)
    assert np.array_equal(m.get_params(), th1)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), tp)
    x = b["states"][:8]
    assert _close(m.forward(x), oracle.deep_forward(bs, C, th1, x))
    snk.update_target_net_(m)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), th1)
    assert np.array_equal(m.forward(x, snk.SNK_NET_TARGET), m.forward(x))


def test_deep_training_batch_bound(snk):
    """The bf16 backward is built for B = 64 batches (its chunk slabs grow with B,
    conv_dx puts B on grid.y): a training batch past the library's bound fails
    cleanly with SNK_ERR_INVALID before any allocation or launch."""
    rb = _replay(snk, 10, 2, n=64, T=130)
    m = snk.DQNModel(10, 3, n_frames=2, seed=2, deep=True)
    ids = snk.DeviceArray(8193, np.int64)
    ids.upload(np.arange(8193, dtype=np.int64))
    with pytest.raises(snk.SnakeHipError, match="training batch"):
        m.loss_grad(rb, ids, 8193)


def test_deep_trainer_graph_vs_eager_and_counts(snk):
    """The batched train! loop with the deep net (64 envs of 10x10): the
    graph-replayed and eager runs give identical parameters and losses, with
    the reference's update count and epsilon schedule."""
    outs = []
    for graph in (True, False):
        tr = snk.Trainer(n_envs=64, board_size=10, n_frames=2, capacity=500, n_batches=9, target_update_rate=4,
                         decay=1e-2, seed=5, deep=True)
        st = snk.train_(tr, graph=graph)
        outs.append((tr.model.get_params(), tr.model.get_params(snk.SNK_NET_TARGET), tr.losses, st))
    (p0, t0, l0, s0), (p1, t1, l1, s1) = outs
    assert np.array_equal(p0, p1) and np.array_equal(t0, t1) and np.array_equal(l0, l1)
    assert s0["updates"] == 10 and len(l0) == 10 and np.all(np.isfinite(l0))
    eps = np.float32(1.0)
    for _ in range(10):
        eps = max(np.float32(eps - np.float32(1e-2)), np.float32(0.05))
    assert np.float32(s0["epsilon"]) == eps


def test_configs2_act_forward_65536_envs(snk):
    """configs[2] at size: 65,536 lockstep 20x20 envs, 2 frames: the deep
    net's epsilon-greedy forward over every env state; 64 states spread over
    the batch within the Q tolerance of the oracle, and greedy actions its
    first argmax wherever the top-2 margin exceeds 1e-3."""
    n, bs, C = 65536, 20, 2
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    act = snk.DeviceArray(n, np.uint8)
    for _ in range(12):
        snk.synth_actions_dev(g, 202, act)
        snk.step_indices_dev(g, act.ptr)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=31, deep=True)
    p = _scaled(m, np.random.default_rng(1))
    q = m.q_env(g)
    a = snk.epsilon_greedy(g, m, 0.0)
    x = snk.assemble_state_(g)
    sel = np.linspace(0, n - 1, 64).astype(np.int64)
    qref = oracle.deep_forward(bs, C, p, x[sel])
    print(f"configs[2] act forward: err {_err(q[sel], qref):.2e}, |Q| max {np.abs(qref).max():.2f}")
    assert _close(q[sel], qref), _err(q[sel], qref)
    top = np.sort(qref, axis=1)
    ok = top[:, 2] - top[:, 1] > 1e-3
    ref_a = np.argmax(qref, axis=1)
    assert ok.sum() > 40 and np.array_equal(a[sel][ok], ref_a[ok])


def test_deep_net_refused_by_jacobian_and_laplace_sampling(snk):
    """The per-sample Jacobian, the Jacobian Gram and laplace_sampling! run the
    reference architecture's kernels: a deeper-net handle is refused with
    SnakeHipError (no fault, no silent wrong answer)."""
    m = snk.DQNModel(12, 3, n_frames=2, seed=3, deep=True)
    rb = snk.ReplayBuffer(256, board_size=12, n_frames=2, batch_size=64)
    g = snk.SnakeGame(12, 2, n_envs=64, autoreset=True)
    act = snk.DeviceArray(64, np.uint8)
    for _ in range(4):
        snk.synth_actions_dev(g, 1, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    with pytest.raises(snk.SnakeHipError, match="deep"):
        snk.jacobian(m, rb, 8)
    with pytest.raises(snk.SnakeHipError, match="deep"):
        snk.jacobian_gram(m, rb, 128)
    lap = snk.LaplaceD(m.P, 3)
    for k in range(3):
        lap.snapshot(m, k)
    lap.fit_center()
    tr = snk.Trainer(n_envs=64, board_size=12, n_frames=2, capacity=256, model=m, seed=3)
    with pytest.raises(snk.SnakeHipError, match="deep"):
        snk.laplace_sampling_(tr, lap, n_models=4)


def _threaded(fn, parts, workers=16):
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(workers, len(parts))) as ex:
        return list(ex.map(fn, parts))


def _deep_q(bs, C, p, x):
    parts = [ix for ix in np.array_split(np.arange(len(x)), min(16, len(x))) if len(ix)]
    return np.concatenate(_threaded(lambda ix: oracle.deep_forward(bs, C, p, x[ix]), parts))


def _deep_loss_grad(bs, C, qp, tp, f, ac, rw, dn, mk):
    """oracle.deep_loss_grad over the batch in 16 threads: the Huber loss is a mean, so the
    chunks' (loss, gradient) are weighted by their share of the batch (fp64 sums)."""
    B = len(ac)
    parts = [ix for ix in np.array_split(np.arange(B), 16) if len(ix)]
    res = _threaded(lambda ix: oracle.deep_loss_grad(bs, C, qp, tp, f[ix, :C], ac[ix], rw[ix], f[ix, 1:], dn[ix],
                                                     mk[ix]), parts)
    loss = sum(r[0] * len(ix) for r, ix in zip(res, parts)) / B
    g = sum(r[1] * len(ix) for r, ix in zip(res, parts)) / B
    return loss, g


def test_configs2_trainer_graph_trajectory_vs_oracle(snk):
    """configs[2] as bench.py times it: 65,536 lockstep 20x20 games, 2 frames, the
    deeper bf16 net, replay capacity 50,000 (each lockstep step overfills it: only the
    step's last 50,000 transitions survive, as sequential store! leaves them), B = 64,
    one captured graph of 4 iterations (deep_front_kernel / deep_conv3_kernel /
    deep_dense1_ldsb_kernel act forward over 65,536 states, the 20x20 step + store, the
    deep update: deep_conv3_small_kernel forward, the LDS-image backward kernels,
    RMSProp + images + target sync). epsilon 0.25, so most actions are greedy.
    The act / Q trace and the gradient trace make every iteration of the graph
    observable; the oracle replays it decision by decision:
      explored actions, env outputs, boards, all 50,000 replay slots   bit-exact
      greedy actions == first argmax of the device's own Q            exact
      Q of 96 sampled states per iteration (every part of the grid)
        vs the oracle's bf16 restatement at that iteration's params   2e-3 (as above)
      greedy actions vs the oracle argmax (top-2 margin > 1e-3)       exact
      every update, teacher-forced (the device's q_net, t_net, accumulator before it):
        loss relative 2e-3, gradient normwise 1e-3
      q_net, accumulator, t_net after the graph == Float32 RMSProp of the traced
        gradients, t_net synced at nb % 3 == 0                        bit-exact"""
    from devrng import TRAINER_SAMPLE_SALT, explore_np, first_argmax_np, floyd
    bs, C, n, cap, B, rate, U, eps, seed = 20, 2, 65536, 50_000, 64, 3, 4, np.float32(0.25), 0xD2D2
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=cap, batch_size=B, n_batches=10_000,
                     target_update_rate=rate, epsilon=float(eps), epsilon_end=float(eps), decay=0.0, seed=seed,
                     graph_unroll=U, deep=True)
    m = tr.model
    P = m.P
    perm = m.flux_index()
    gring = snk.DeviceArray((U, P), np.float32)
    aring = snk.DeviceArray((U, n), np.uint8)
    qring = snk.DeviceArray((U, n, 3), np.float32)
    tr.set_trace(gring)
    tr.set_act_trace(aring, qring)
    ob = oracle.OracleBatch(n, bs, C)
    nc = bs * bs
    frames = np.zeros((cap, C + 1, nc), np.int8)
    o_act = np.zeros(cap, np.int32)
    o_rew = np.zeros(cap, np.float32)
    o_done = np.zeros(cap, np.uint8)
    o_mask = np.zeros((cap, 3), np.uint8)
    st = {"count": 0, "t": 0, "q": 0.0, "greedy": 0}

    def check_acts(a, q, th, it):
        states = ob.states()
        ex = explore_np(seed, n, st["t"], eps)
        rnd = ex >= 0
        assert np.array_equal(a[rnd], ex[rnd]), st["t"]
        assert np.array_equal(a[~rnd], first_argmax_np(q[~rnd])), st["t"]
        sel = np.linspace(0, n - 8, 96).astype(np.int64) + it % 7
        qref = _deep_q(bs, C, th, states[sel].astype(np.float32))
        err = _err(q[sel], qref)
        st["q"] = max(st["q"], err)
        assert err <= 2e-3, (st["t"], err)
        g = ~rnd[sel]
        top = np.sort(qref[g], axis=1)
        ok = top[:, 2] - top[:, 1] > 1e-3
        assert np.array_equal(a[sel][g][ok], first_argmax_np(qref[g])[ok]), st["t"]
        st["greedy"] += int(ok.sum())

    def oracle_step(a):
        out = ob.step(a)
        keep = np.arange(max(0, n - cap), n)           # the step's surviving transitions
        k = (st["count"] + keep) % cap
        frames[k], o_act[k], o_rew[k] = out["frames"][keep], a[keep], out["reward"][keep]
        o_done[k], o_mask[k] = out["done"][keep], out["mask"][keep]
        st["count"] += n
        st["t"] += 1
        return out

    def check_env(out):
        o = tr.game.last("reward", "done", "mask")
        assert np.array_equal(o["reward"], out["reward"]) and np.array_equal(o["done"], out["done"]), st["t"]
        assert np.array_equal(o["mask"], out["mask"] @ np.array([1, 2, 4], np.uint8)), st["t"]
        assert np.array_equal(tr.game.board_cells(), ob.boards()), st["t"]

    th0 = m.get_params()
    tr.run(1, learn=False, graph=True)                   # fill_buffer!: one step overfills the ring
    check_acts(aring.numpy()[0], qring.numpy()[0], th0, 0)
    out = oracle_step(aring.numpy()[0])
    check_env(out)
    assert len(tr.buffer) == cap

    th, acc, tt = m.get_params(), m.get_params(snk.SNK_NET_OPT_STATE), m.get_params(snk.SNK_NET_TARGET)
    tr.run(U, learn=True, graph=True)
    acts, qs = aring.numpy(), qring.numpy()
    gdev = np.empty((U, P), np.float32)
    gdev[:, perm] = gring.numpy()
    losses = tr.losses
    sseed = seed ^ TRAINER_SAMPLE_SALT
    worst_l = worst_g = 0.0
    for i in range(U):
        check_acts(acts[i], qs[i], th, 1 + i)
        out = oracle_step(acts[i])
        ids = floyd(sseed, i, min(st["count"], cap), B)
        f = frames[ids]
        lref, gref = _deep_loss_grad(bs, C, th, tt, f, o_act[ids], o_rew[ids], o_done[ids], o_mask[ids])
        rl = abs(losses[i] - lref) / abs(lref)
        rg = float(np.linalg.norm(gdev[i] - gref) / np.linalg.norm(gref))
        worst_l, worst_g = max(worst_l, rl), max(worst_g, rg)
        assert rl <= 2e-3 and rg <= 1e-3, (i, rl, rg)
        th, acc = oracle.rmsprop(th, acc, gdev[i])
        if i % rate == 0:
            tt = th.copy()
    check_env(out)
    assert np.array_equal(m.get_params(), th) and np.array_equal(m.get_params(snk.SNK_NET_OPT_STATE), acc)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), tt)
    s = tr.stats()
    assert s["updates"] == U and s["env_steps"] == st["t"] * n
    got = snk.stack_exp(tr.buffer, np.arange(cap))
    assert np.array_equal(got["states"], frames[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], frames[:, 1:].astype(np.float32))
    assert np.array_equal(got["actions"], o_act + 1) and np.array_equal(got["rewards"], o_rew)
    assert np.array_equal(got["dones"], o_done.astype(bool))
    assert np.array_equal(got["suicidal_mask"], o_mask.astype(bool))
    print(f"configs[2] graph: {st['t']} steps of {n} envs, Q max err {st['q']:.2e}, {st['greedy']} greedy actions "
          f"vs the oracle; {U} updates: loss rel max {worst_l:.2e}, gradient max {worst_g:.2e}")
