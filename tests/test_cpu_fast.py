"""The CPU baseline (oracle/cpu_fast.cpp, what bench.py times as
cpu_baseline) computes the same thing as the oracle: env bit-exact, Q-values
and the DQN gradient within fp32 error (1e-5 relative). CPU only."""
import numpy as np
import pytest

import oracle


@pytest.mark.parametrize("bs,C", [(10, 2), (12, 1), (12, 2)])
def test_cpu_fast_env_bitexact_vs_oracle(bs, C):
    L = oracle.fast()
    n, T = 64, 300
    food, _ = oracle.food_list(bs)
    h = L.cpuf_env_create(n, bs, C, 500, food, len(food))
    ob = oracle.OracleBatch(n, bs, C)
    r, d, m = np.zeros(n, np.float32), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    boards = np.zeros((n, bs * bs), np.int8)
    for t in range(T):
        a = oracle.synth_actions(0xFA57 + bs, n, t)
        L.cpuf_env_step(h, a, r, d, m, 4)
        ref = ob.step(a, want_frames=False)
        assert np.array_equal(r, ref["reward"]) and np.array_equal(d, ref["done"]), t
        assert np.array_equal(m, ref["mask"] @ np.array([1, 2, 4], np.uint8)), t
    L.cpuf_env_boards(h, boards)
    assert np.array_equal(boards, ob.boards())
    L.cpuf_env_destroy(h)


@pytest.mark.parametrize("bs,C", [(10, 2), (12, 1)])
def test_cpu_fast_forward_and_loss_grad_vs_oracle(bs, C):
    L = oracle.fast()
    rng = np.random.default_rng(bs)
    P = oracle.qnet_nparams(bs, C)
    p = (rng.standard_normal(P) * 0.05).astype(np.float32)
    tp = (p + rng.standard_normal(P).astype(np.float32) * np.float32(0.01)).astype(np.float32)
    B = 12
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    q = np.zeros((B, 3), np.float32)
    L.cpuf_qnet_forward(bs, C, p, B, x, q, 4)
    qref = oracle.qnet_forward(bs, C, p, x)
    assert np.all(np.abs(q - qref) <= 1e-5 * np.maximum(1.0, np.abs(qref)))
    sn = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    a = rng.integers(0, 3, B).astype(np.int32)
    r = rng.standard_normal(B).astype(np.float32)
    d = rng.integers(0, 2, B).astype(np.uint8)
    m3 = rng.integers(0, 2, (B, 3)).astype(np.uint8)
    g = np.zeros(P, np.float32)
    loss = L.cpuf_loss_grad(bs, C, p, tp, B, x, a, r, sn, d, m3, g, 4)
    lref, gref, _ = oracle.dqn_loss_grad(bs, C, p, tp, x, a, r, sn, d, m3)
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    assert np.linalg.norm(g - gref) <= 1e-5 * np.linalg.norm(gref)
