"""GPU parity of the Laplace D build against the oracle.

  snapshots           D[:, pos] == Float64.(theta) bit-exact (compute_D.jl:70)
  Welford + centring  mean, var and the centred D bit-exact (fp64, the
                      reference's operation order, compute_D.jl:21-27, 80-81)
  Gram D'D            |G - G_ref| <= 1e-5 * sqrt(G_ii G_jj) (fp32 MFMA over
                      the fp32-rounded centred D, fp64 accumulation)
  Jacobian rows       ||J_s - J_ref,s|| <= 1e-5 ||J_ref,s|| and per element
                      |dJ| <= 1e-5 * max|J_ref,s| + 1e-4 |J_ref,s|
  Jacobian Gram J J'  |G - G_ref| <= 1e-5 * sqrt(G_ii G_jj), exactly symmetric

The Jacobian has no reference counterpart (the reference's
D is snapshot-based), so its oracle is the restated backward
(oracle/snake_oracle.c orc_qnet_backward, pinned only through the loss
gradient path): parity unpinned against the reference itself.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _replay(snk, bs, C, n=64, T=12, seed=5):
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * T, board_size=bs, n_frames=C, batch_size=64)
    act = snk.DeviceArray(n, np.uint8)
    for _ in range(T):
        snk.synth_actions_dev(g, seed, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    return g, rb


def _gram_close(G, Gref, tol=1e-5):
    d = np.sqrt(np.clip(np.diag(Gref), 0, None))
    scale = np.outer(d, d) + 1e-30
    return float(np.max(np.abs(G - Gref) / scale))


@pytest.mark.parametrize("K,P", [(37, 1001), (130, 4099)])
def test_welford_center_bitexact(snk, K, P):
    rng = np.random.default_rng(K)
    base = rng.standard_normal(P) * 0.3
    D0 = base[None, :] + rng.standard_normal((K, P)) * 1e-3   # snapshots around a mean, as in training
    lap = snk.LaplaceD(P, K)
    for k in range(K):
        lap.set_column(k, D0[k])
    lap.fit_center()
    Dref, mref, vref = oracle.welford_center(D0)
    assert np.array_equal(lap.mean(), mref)
    assert np.array_equal(lap.var(), vref)
    assert np.array_equal(lap.D(), Dref)


def test_snapshot_flux_order(snk):
    m = snk.DQNModel(12, 3, n_frames=2, seed=9)
    theta = m.get_params()
    lap = snk.LaplaceD(m.P, 3)
    lap.snapshot(m, 1)
    D = lap.D()
    assert np.array_equal(D[1], theta.astype(np.float64))
    assert not D[0].any() and not D[2].any()   # zeros(Float64, (P, K))


@pytest.mark.parametrize("K,P", [(130, 5003), (300, 20000)])
def test_gram_vs_oracle(snk, K, P):
    rng = np.random.default_rng(P)
    D0 = rng.standard_normal((K, P)) * 1e-2 + rng.standard_normal(P)[None, :]
    lap = snk.LaplaceD(P, K)
    for k in range(K):
        lap.set_column(k, D0[k])
    lap.fit_center()
    G, ms = lap.gram()
    Dc, _, _ = oracle.welford_center(D0)
    Gref = Dc @ Dc.T
    assert np.array_equal(G, G.T)
    assert _gram_close(G, Gref) <= 1e-5
    lam = lap.spectrum(G)
    assert lam.size > 0 and np.all(lam > 0)


def test_gram_matches_restated_oracle_small(snk):
    rng = np.random.default_rng(1)
    D0 = rng.standard_normal((20, 333))
    lap = snk.LaplaceD(333, 20)
    for k in range(20):
        lap.set_column(k, D0[k])
    lap.fit_center()
    G, _ = lap.gram()
    Dc, _, _ = oracle.welford_center(D0)
    assert _gram_close(G, oracle.gram(Dc)) <= 1e-5


def _oracle_jacobian(bs, C, params, states, a_idx):
    J = np.zeros((len(a_idx), params.size), np.float64)
    for s, a in enumerate(a_idx):
        dq = np.zeros((1, 3))
        dq[0, a] = 1.0
        J[s] = oracle.qnet_backward(bs, C, params, states[s:s + 1], dq)
    return J


@pytest.mark.parametrize("bs,C", [(12, 2), (10, 1)])
def test_jacobian_rows_vs_oracle(snk, bs, C):
    _, rb = _replay(snk, bs, C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=17)
    slots = np.array([0, 5, 17, 63, 64, 200, 511, 767], np.int64)
    J = snk.jacobian(m, rb, slots=slots)
    b = snk.stack_exp(rb, slots)
    Jref = _oracle_jacobian(bs, C, m.get_params(), b["states"], (b["actions"] - 1) % 3)
    for s in range(len(slots)):
        r, rr = J[s].astype(np.float64), Jref[s]
        assert np.linalg.norm(r - rr) <= 1e-5 * np.linalg.norm(rr), s
        assert np.all(np.abs(r - rr) <= 1e-5 * np.abs(rr).max() + 1e-4 * np.abs(rr)), s


@pytest.mark.parametrize("bs,C,n", [(12, 2, 300), (10, 1, 129)])
def test_jacobian_gram_vs_oracle(snk, bs, C, n):
    _, rb = _replay(snk, bs, C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=23)
    G, ms = snk.jacobian_gram(m, rb, n)
    assert len(ms) == 4 and all(t >= 0 for t in ms)
    assert np.array_equal(G, G.T)
    b = snk.stack_exp(rb, np.arange(n))
    Jref = _oracle_jacobian(bs, C, m.get_params(), b["states"], (b["actions"] - 1) % 3)
    Gref = Jref @ Jref.T
    assert _gram_close(G.astype(np.float64), Gref) <= 1e-5


def test_jacobian_gram_matches_device_jacobian(snk):
    """Larger n: the decomposed Gram equals the Gram of the materialised
    device Jacobian (size-independent consistency of the two paths)."""
    bs, C, n = 12, 2, 700
    _, rb = _replay(snk, bs, C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=29)
    G, _ = snk.jacobian_gram(m, rb, n)
    J = snk.jacobian(m, rb, n).astype(np.float64)
    Gref = J @ J.T
    assert _gram_close(G.astype(np.float64), Gref) <= 2e-6


def test_spectrum_ncols_and_trajectory_match_svd(snk):
    """plot_traj.jl's analysis from the device Gram equals numpy's svd of the
    (oracle-)centred D: eigenvalues S^2/(K-1), compute_n_cols, and the 2-D
    trajectory U[:, 1:2]' D (up to the sign of each singular vector)."""
    K, P = 60, 3000
    rng = np.random.default_rng(7)
    D0 = rng.standard_normal(P)[None, :] + np.cumsum(rng.standard_normal((K, P)) * 1e-2, axis=0)
    lap = snk.LaplaceD(P, K)
    for k in range(K):
        lap.set_column(k, D0[k])
    lap.fit_center()
    Dc, _, _ = oracle.welford_center(D0)
    U, S, Vt = np.linalg.svd(Dc.T, full_matrices=False)   # Julia's D is P x K
    lam_ref = S ** 2 / (K - 1)
    lam, _ = lap.eig()
    assert np.allclose(lam[:10], lam_ref[:10], rtol=1e-5)
    assert snk.LaplaceD.n_cols(lam) == snk.LaplaceD.n_cols(lam_ref)
    Y = lap.trajectory_2d()
    Yref = U[:, :2].T @ Dc.T
    for i in range(2):
        sgn = np.sign(np.dot(Y[i], Yref[i]))
        assert np.allclose(sgn * Y[i], Yref[i], rtol=1e-4, atol=1e-6 * np.abs(Yref[i]).max())
