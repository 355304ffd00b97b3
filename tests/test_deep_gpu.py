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
