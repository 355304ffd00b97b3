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


def test_gram_reference_scale_entrywise(snk):
    """plot_traj.jl:10-16 at compute_D.jl's own size: K = 1000 snapshots of
    the 12x12 net (P = 279,699). The snapshots are a training-like
    trajectory (a random walk around theta_0 plus per-snapshot jitter), so the
    centred Gram has large off-diagonal entries of both signs. Checked against
    fp64 Dc Dc' of the oracle's centred D (itself bit-exact with the device's):
    every entry |G - G_ref| <= 1e-5 sqrt(G_ii G_jj), and every entry with
    |G_ref| >= 0.01 sqrt(G_ii G_jj) also relative <= 1e-5."""
    K, P = 1000, 279_699
    rng = np.random.default_rng(1000)
    D0 = rng.standard_normal((K, P), dtype=np.float32).astype(np.float64)
    D0 *= 2e-4
    np.cumsum(D0, axis=0, out=D0)                                  # the walk
    D0 += rng.standard_normal((K, P), dtype=np.float32) * 1e-4     # jitter
    D0 += rng.standard_normal(P, dtype=np.float32)[None, :] * 0.05  # theta_0
    lap = snk.LaplaceD(P, K)
    for k in range(K):
        lap.set_column(k, D0[k])
    lap.fit_center()
    G, ms = lap.gram()
    Dc, _, _ = oracle.welford_center(D0)
    del D0
    assert np.array_equal(lap.D(), Dc)
    Gref = Dc @ Dc.T
    d = np.sqrt(np.diag(Gref))
    scale = np.outer(d, d)
    err = np.abs(G - Gref)
    big = np.abs(Gref) >= 0.01 * scale
    rel = err[big] / np.abs(Gref[big])
    print(f"D'D K={K} P={P}: max normalised err {float((err / scale).max()):.2e}; {int(big.sum())} of {K * K} "
          f"entries >= 0.01 sqrt(GiiGjj): max rel {rel.max():.2e}, median {np.median(rel):.2e}; "
          f"{int((Gref < 0).sum())} negative; kernel {ms:.2f} ms")
    assert np.array_equal(G, G.T)
    assert float((err / scale).max()) <= 1e-5
    assert big.sum() > K * K // 2 and (Gref[big] < 0).sum() > 1000 and rel.max() <= 1e-5


def test_gram_ksplit_and_x6_slab_paths(snk):
    """compute_D.jl's D'D on the production path (fit_center splits the centred rows into h3
    planes, one power-of-two exponent per row and 1024-column chunk; syrk_h3k_kernel's fp32 chunk
    partials summed in fp64 by syrk_ksum_kernel) and on the round-5 x6 slab kernel
    (snk.arith(syrk_ksplit=False)): both within 1e-5 sqrt(G_ii G_jj) of the fp64 oracle, exactly
    symmetric, the centred D bit-identical either way. K = 300 snapshots over two 256-row
    blocks (a partial tile), P = 20,000 (a partial last chunk)."""
    K, P = 300, 20_000
    rng = np.random.default_rng(11)
    D0 = rng.standard_normal((K, P)) * 1e-2 + rng.standard_normal(P)[None, :]
    Dc, _, _ = oracle.welford_center(D0)
    Gref = Dc @ Dc.T
    out = {}
    for ks in (True, False):
        with snk.arith(syrk_ksplit=ks):
            lap = snk.LaplaceD(P, K)
            for k in range(K):
                lap.set_column(k, D0[k])
            lap.fit_center()
            assert np.array_equal(lap.D(), Dc)
            G, _ = lap.gram()
        assert np.array_equal(G, G.T)
        out[ks] = _gram_close(G, Gref)
        assert out[ks] <= 1e-5, (ks, out[ks])
    print(f"D'D normalised max error: k-split h3 {out[True]:.2e}, x6 slab {out[False]:.2e}")


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


# ---------------------------------------------------------------- Laplace sampling (la_utils.jl:83-118)
def _fitted_lap(snk, m, K, seed=0, spread=0.02):
    """K q_net snapshots spread around m's weights, Welford-fitted and centred."""
    rng = np.random.default_rng(seed)
    p0 = m.get_params()
    lap = snk.LaplaceD(m.P, K)
    for k in range(K):
        m.set_params((p0 + rng.standard_normal(p0.size).astype(np.float32) * np.float32(spread)).astype(np.float32))
        lap.snapshot(m, k)
    m.set_params(p0)
    lap.fit_center()
    return lap


def test_laplace_normals_stream(snk):
    """The z stream of sample_model: N(0, 1) moments (5-sigma bounds on
    200k draws), streams 1 and 2 and different models independent, and
    index-addressable (a sub-range equals the same indices of a longer draw)."""
    z = snk.laplace_normals(5, 3, 1, 0, 200_000)
    assert abs(z.mean()) < 5 / np.sqrt(z.size) and abs(z.var() - 1) < 5 * np.sqrt(2 / z.size)
    assert abs(np.mean(z ** 4) - 3) < 0.1 and np.all(np.isfinite(z))
    z2 = snk.laplace_normals(5, 3, 2, 0, 200_000)
    z_other = snk.laplace_normals(5, 4, 1, 0, 200_000)
    assert abs(np.corrcoef(z, z2)[0, 1]) < 0.02 and abs(np.corrcoef(z, z_other)[0, 1]) < 0.02
    assert np.array_equal(snk.laplace_normals(5, 3, 1, 1000, 500), z[1000:1500])


def test_sample_model_bitexact_vs_restatement(snk):
    """sample_model (la_utils.jl:83-95) given the device z: the numpy
    restatement of w = mean + 1/sqrt(2) sqrt|var| z1 + 1/sqrt(2(K-1)) D z2
    (Float64, term by term, the D*z2 sum k-ascending) rounds to the same
    Float32 weights bit for bit (Flux order)."""
    bs, C, K = 10, 2, 7
    m = snk.DQNModel(bs, 3, n_frames=C, seed=3)
    lap = _fitted_lap(snk, m, K)
    D, mean, var = lap.D(), lap.mean(), lap.var()       # D: [K][P] (Julia's P x K)
    for n in (0, 11):
        w = snk.sample_model(lap, m, n=n, seed=9)
        z1 = snk.laplace_normals(9, n, 1, 0, m.P)
        z2 = snk.laplace_normals(9, n, 2, 0, K)
        c1, c2 = 1.0 / np.sqrt(2.0), 1.0 / np.sqrt(2.0 * (K - 1))
        d = np.zeros(m.P)
        for k in range(K):
            d = d + (c2 * D[k]) * z2[k]
        ref = ((mean + (c1 * np.sqrt(np.abs(var))) * z1) + d).astype(np.float32)
        assert np.array_equal(w, ref), np.abs(w - ref).max()


def _oracle_greedy_episode(bs, C, params):
    """play_episode(model, 0f0) on the CPU oracle: fp64 forward, first-max
    argmax, oracle step!; returns (Float32 reward, length, min top-2 margin)."""
    ob = oracle.OracleBatch(1, bs, C)
    ep, L, margin = np.float32(0), 0, np.inf
    while True:
        q = oracle.qnet_forward(bs, C, params, ob.states().astype(np.float32))[0]
        srt = np.sort(q)
        margin = min(margin, float(srt[-1] - srt[-2]) / max(1.0, abs(float(srt[-1]))))
        r = ob.step(np.array([int(np.argmax(q))], np.uint8), want_frames=False)
        ep = np.float32(ep + np.float32(r["reward"][0]))
        L += 1
        if r["done"][0]:
            return float(ep), L, margin


def test_laplace_sampling_lockstep_episodes(snk):
    """laplace_sampling! (la_utils.jl:97-118) with 6 models in chunks of 4:
    every model's lockstep greedy episode (per-env-weights forward) has the
    reward and length of play_episode(re(w), 0f0) on the CPU oracle (fp64
    forward + step!) whenever no step's top-2 Q margin is below 1e-4
    (relative); tr_reward is tr.model's greedy episode on the oracle; the
    buffer grows by exactly the better models' transitions, appended in
    (model, step) order (their rewards sum to the models' episode rewards)."""
    bs, C, K = 10, 2, 5
    tr = snk.Trainer(n_envs=1, board_size=bs, n_frames=C, capacity=20000, seed=5)
    lap = _fitted_lap(snk, tr.model, K, seed=1)
    before = len(tr.buffer)
    res = snk.laplace_sampling_(tr, lap, n_models=6, seed=13, chunk=4)
    ref_r, ref_l, ref_m = _oracle_greedy_episode(bs, C, tr.model.get_params())
    if ref_m > 1e-4:
        assert res["tr_reward"] == np.float32(ref_r)
    checked = 0
    for n in range(6):
        w = snk.sample_model(lap, tr.model, n=n, seed=13)
        r, L, margin = _oracle_greedy_episode(bs, C, w)
        if margin > 1e-4:
            assert res["rewards"][n] == np.float32(r) and res["lengths"][n] == L, (n, res["rewards"][n], r)
            checked += 1
    assert checked >= 3
    better = [n for n in range(6) if res["rewards"][n] > res["tr_reward"]]
    assert res["n_better_models"] == len(better)
    grown = int(sum(res["lengths"][n] for n in better))
    assert len(tr.buffer) == before + grown
    if grown:
        got = snk.stack_exp(tr.buffer, np.arange(before, before + grown, dtype=np.int64))
        o = 0
        for n in better:
            L = int(res["lengths"][n])
            s = np.float32(0)
            for v in got["rewards"][o:o + L]:
                s = np.float32(s + np.float32(v))
            assert s == res["rewards"][n] and got["dones"][o + L - 1]
            o += L


def test_laplace_sampling_wraps_small_buffer(snk):
    """More better-model transitions than the buffer holds: store! in
    (model, step) order keeps exactly the last `capacity` of them, each in the
    ring slot the sequential stores leave it in, and the count advances by all
    of them (utils.jl:267-277). Checked against the same sampling into a
    buffer large enough to hold everything."""
    bs, C, K, cap = 10, 2, 5, 8
    big = snk.Trainer(n_envs=1, board_size=bs, n_frames=C, capacity=20000, seed=5)
    small = snk.Trainer(n_envs=1, board_size=bs, n_frames=C, capacity=cap, batch_size=4, seed=5)
    # tr.model always takes action index 0 (Dense2 = 0, bias (1, 0, 0)): straight up
    # into the wall, 7 steps and reward -1.06; sampled models that die sooner beat it
    p = big.model.get_params()
    p[-195:] = 0
    p[-3] = 1
    for t in (big, small):
        t.model.set_params(p)
    lap = _fitted_lap(snk, big.model, K, seed=1, spread=0.5)
    c0 = 3                                   # a partly filled ring to start from
    fr = np.zeros((c0, C + 1, bs * bs), np.int8)
    snk.store_(small.buffer, fr, np.zeros(c0), np.zeros(c0, np.float32), np.zeros(c0), np.zeros((c0, 3)),
               np.zeros(c0))
    rb = snk.laplace_sampling_(big, lap, n_models=32, seed=21, chunk=16)
    rs = snk.laplace_sampling_(small, lap, n_models=32, seed=21, chunk=16)
    assert rs["n_better_models"] == rb["n_better_models"]
    grown = len(big.buffer)
    assert grown > cap, "the sampling must overflow the small ring for this test"
    assert small.buffer.count == c0 + grown and len(small.buffer) == cap
    ref = snk.stack_exp(big.buffer, np.arange(grown - cap, grown))
    slots = (c0 + np.arange(grown - cap, grown)) % cap
    got = snk.stack_exp(small.buffer, slots)
    for k in ("states", "next_states", "actions", "rewards", "dones", "suicidal_mask"):
        assert np.array_equal(got[k], ref[k]), k


def test_jacobian_gram_shards_reassemble_bitexact(snk):
    """D(50k) across ranks, one device: the three shards of a 3-rank split,
    each into its own zeroed G, hold disjoint tiles (+ mirror) whose sum is
    the single-launch Gram bit for bit (a tile's arithmetic does not depend on
    which launch computes it); n = 700 leaves a partial last tile row."""
    bs, C, n = 12, 2, 700
    _, rb = _replay(snk, bs, C)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=29)
    G, _ = snk.jacobian_gram(m, rb, n)
    total = np.zeros((n, n), np.float64)
    nz = np.zeros((n, n), np.int32)
    for r in range(3):
        Gr = snk.DeviceArray((n, n), np.float32)
        Gr.zero()
        snk.jacobian_gram_shard(m, rb, n, r, 3, Gr)
        h = Gr.numpy()
        total += h
        nz += (h != 0)
        for i0, j0 in snk.gram_tiles(n, r, 3):
            blk = h[i0:i0 + 128, j0:j0 + 128]
            assert np.array_equal(blk, G[i0:i0 + 128, j0:j0 + 128])
    assert nz.max() <= 1
    assert np.array_equal(total.astype(np.float32), G)
    # a one-rank communicator's gather is the identity
    comm = snk.Comm(1, 0, snk.Comm.unique_id())
    Gd = snk.DeviceArray((n, n), np.float32)
    Gd.upload(G)
    snk.jacobian_gram_gather(comm, n, Gd, 0)
    assert np.array_equal(Gd.numpy(), G)
