"""BASELINE.json's configs exercised at their own sizes on the device.

configs[0]  1 env, 12x12, 1 frame, 1000 mini-batches on the reference's own
            one-episode-per-update schedule (utils.jl:389-482): fill and the
            first updates replayed on the oracle decision by decision.
configs[1]  4096 lockstep 12x12 envs, 2 frames: env + store bit-exact over 100
            steps, the act forward (conv_h3f_kernel path) vs the oracle.
configs[4]  the Jacobian Gram over the full 50,000-transition buffer: sampled
            entries across every tile class vs fp64 dot products of
            oracle-computed Jacobian rows.
(configs[2] is the bf16 deeper net, tested in test_deep_gpu.py; configs[3]
needs the 8-GPU node and is covered by the world-size tests.)

Tolerances are stated in each test.
"""
import numpy as np
import pytest

import oracle
from devrng import explore, first_argmax, floyd

pytestmark = pytest.mark.gpu


def _qclose(q, qref):
    return np.all(np.abs(q - qref) <= 1e-5 * np.maximum(1.0, np.abs(qref)))


def test_configs1_env_4096_store_bitexact(snk):
    """configs[1]: 4096 envs of 12x12, 2 frames, counter-RNG actions,
    100 lockstep steps through the fused step + store! kernel. Every output
    of every step, the boards at three points and 8192 random replay slots
    are bit-exact with the oracle."""
    n, bs, C, T, seed = 4096, 12, 2, 100, 0x4096
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * T, board_size=bs, n_frames=C, batch_size=64)
    ob = oracle.OracleBatch(n, bs, C)
    act = snk.DeviceArray(n, np.uint8)
    rng = np.random.default_rng(0)
    pick = np.sort(rng.choice(n * T, 8192, replace=False))
    ref = {}
    for t in range(T):
        snk.synth_actions_dev(g, seed, act)
        a = act.numpy()
        snk.step_indices_dev(g, act.ptr, replay=rb)
        r = ob.step(a)
        o = g.last()
        assert np.array_equal(o["reward"], r["reward"]) and np.array_equal(o["done"], r["done"]), t
        assert np.array_equal(o["mask"], r["mask"] @ np.array([1, 2, 4], np.uint8)), t
        assert np.array_equal(o["dirs"], r["prev_dir"] | (r["dir"] << 2) | (r["done"] << 4)), t
        if t in (0, 49, T - 1):
            assert np.array_equal(g.board_cells(), ob.boards()), t
        lo, hi = np.searchsorted(pick, [t * n, (t + 1) * n])
        for k in pick[lo:hi]:
            ref[int(k)] = (r["frames"][k - t * n], a[k - t * n], r["reward"][k - t * n])
    got = snk.stack_exp(rb, pick)
    fr = np.stack([ref[int(k)][0] for k in pick])
    assert np.array_equal(got["states"], fr[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], fr[:, 1:].astype(np.float32))
    assert np.array_equal(got["actions"], np.array([ref[int(k)][1] for k in pick], np.int32) + 1)
    assert np.array_equal(got["rewards"], np.array([ref[int(k)][2] for k in pick], np.float32))
    assert g.check_faults() == 0


def test_configs1_act_forward_4096_vs_oracle(snk):
    """configs[1]: Q of all 4096 env states in one act forward (conv1 + conv2 +
    conv3 fused in conv_h3f_kernel, Dense1, head); every 4th state (1024, every
    workgroup slot position) within |q - q_ref| <= 1e-5 max(1, |q_ref|) of
    the fp64 oracle, and epsilon_greedy at epsilon 0 picks the oracle's first
    argmax wherever the top-2 margin exceeds 1e-4."""
    n, bs, C = 4096, 12, 2
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    act = snk.DeviceArray(n, np.uint8)
    for _ in range(30):                      # diverse states
        snk.synth_actions_dev(g, 77, act)
        snk.step_indices_dev(g, act.ptr)
    m = snk.DQNModel(bs, 3, n_frames=C, seed=31)
    q = m.q_env(g)
    a = snk.epsilon_greedy(g, m, 0.0)
    x = snk.assemble_state_(g)
    sel = np.arange(0, n, 4)
    qref = oracle.qnet_forward(bs, C, m.get_params(), x[sel])
    assert _qclose(q[sel], qref), np.abs(q[sel] - qref).max()
    top = np.sort(qref, axis=1)
    ok = top[:, 2] - top[:, 1] > 1e-4
    ref_a = np.array([first_argmax(r) for r in qref])
    assert ok.sum() > 900 and np.array_equal(a[sel][ok], ref_a[ok])


def _oracle_jrows(bs, C, params, states, a_idx):
    J = np.zeros((len(a_idx), params.size), np.float64)
    for s, a in enumerate(a_idx):
        dq = np.zeros((1, 3))
        dq[0, a] = 1.0
        J[s] = oracle.qnet_backward(bs, C, params, states[s:s + 1], dq)
    return J


def test_configs4_jacobian_gram_50k_sampled_entries(snk):
    """configs[4]: G = J J' over all 50,000 transitions of a full buffer
    (12x12, 2 frames). 40 rows x 40 columns of G are read back, chosen to hit
    the first, interior, boundary and last (partial: 50,000 = 390*128 + 80)
    128-row tiles, both triangles (the mirrored half) and the diagonal, and
    compared with fp64 dot products of the oracle's Jacobian rows for those
    samples. Bounds: every entry |G - G_ref| <= 1e-5 sqrt(G_ii G_jj); entries
    with |G_ref| >= 0.01 sqrt(G_ii G_jj) also entrywise-relative <= 1e-5
    (north_star's bar; measured 3.5e-7 max)."""
    bs, C, n_env, T = 12, 2, 5000, 10
    n = n_env * T
    g = snk.SnakeGame(bs, C, n_envs=n_env, autoreset=True)
    rb = snk.ReplayBuffer(n, board_size=bs, n_frames=C, batch_size=64)
    act = snk.DeviceArray(n_env, np.uint8)
    for _ in range(T):
        snk.synth_actions_dev(g, 0x50, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
    assert len(rb) == n
    m = snk.DQNModel(bs, 3, n_frames=C, seed=41)
    G, ms = snk.jacobian_gram(m, rb, n, host=False)
    rows = np.array([0, 1, 63, 127, 128, 129, 255, 256, 1000, 4095, 4096, 12345, 24999, 25000, 25087, 33333,
                     40000, 49791, 49792, 49919, 49920, 49921, 49950, 49999], np.int64)
    rng = np.random.default_rng(3)
    rows = np.unique(np.concatenate([rows, rng.choice(n, 16, replace=False)]))
    cols = np.unique(np.concatenate([rows[::2], rng.choice(n, 28, replace=False), [0, 127, 49920, 49999]]))
    Gs = np.zeros((len(rows), n), np.float32)
    from snake_amd import _lib
    for r, i in enumerate(rows):
        _lib.call("snk_memcpy_d2h", Gs[r].ctypes.data_as(_lib.vp), _lib.vp(G.ptr.value + int(i) * n * 4), n * 4)
    Gsub = Gs[:, cols].astype(np.float64)
    allid = np.unique(np.concatenate([rows, cols]))
    b = snk.stack_exp(rb, allid)
    J = _oracle_jrows(bs, C, m.get_params(), b["states"], (b["actions"] - 1) % 3)
    pos = {int(s): k for k, s in enumerate(allid)}
    Jr, Jc = J[[pos[int(i)] for i in rows]], J[[pos[int(j)] for j in cols]]
    Gref = Jr @ Jc.T
    dr, dc = np.sqrt((Jr * Jr).sum(1)), np.sqrt((Jc * Jc).sum(1))
    scale = np.outer(dr, dc)
    err = np.abs(Gsub - Gref)
    norm_err = float((err / scale).max())
    big = np.abs(Gref) >= 0.01 * scale
    rel = err[big] / np.abs(Gref[big])
    print(f"D(50k) sampled {Gref.size} entries: max normalised err {norm_err:.2e}; "
          f"{big.sum()} entries >= 0.01 sqrt(GiiGjj): max rel {rel.max():.2e}, median {np.median(rel):.2e}; "
          f"phases ms {[round(t, 1) for t in ms]}")
    assert norm_err <= 1e-5
    assert big.sum() > 100 and rel.max() <= 1e-5
    # the mirror: G[j, i] == G[i, j] bit for bit for the sampled pairs
    for r, i in enumerate(rows[:8]):
        for j in cols[:8]:
            v = np.zeros(1, np.float32)
            _lib.call("snk_memcpy_d2h", v.ctypes.data_as(_lib.vp), _lib.vp(G.ptr.value + (int(j) * n + int(i)) * 4), 4)
            assert v[0] == Gs[r, j]


def test_configs0_episode_schedule_1env_12x12_1frame(snk):
    """configs[0]: Trainer(n_batches=999), one env of 12x12 and 1 frame on the
    reference's schedule: fill_buffer! (episodes until > 50,000 transitions),
    then per nb one epsilon-greedy episode stored + one B=64 update, target
    sync at nb % 1000 == 0, epsilon decay 1e-6 per update. The fill (every
    action, every replay slot) is bit-exact with the oracle replaying the same
    counter-RNG decisions; the first 6 updates' episodes, batches and losses
    (relative 1e-5 at the oracle's own parameters) and the parameters after
    them (normwise 1e-4 of the change) follow the oracle; all 1000 updates run
    with finite losses and the reference's epsilon."""
    from oracle_loops import OracleEpisodeLoop
    from snake_amd.trainer import EpisodeLoop
    bs, C, cap, seed, K = 12, 1, 50_000, 0xF00D, 6
    tr = snk.Trainer(n_envs=1, board_size=bs, n_frames=C, capacity=cap, n_batches=999, seed=seed)
    m = tr.model
    th0 = m.get_params()
    loop = EpisodeLoop(tr)
    played = loop.fill()
    ol = OracleEpisodeLoop(bs, C, cap, seed, th0)
    assert ol.fill() == played and len(tr.buffer) == cap
    got = snk.stack_exp(tr.buffer, np.arange(cap))
    assert np.array_equal(got["states"], ol.frames[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], ol.frames[:, 1:].astype(np.float32))
    assert np.array_equal(got["actions"], ol.act + 1) and np.array_equal(got["rewards"], ol.rew)
    assert np.array_equal(got["dones"], ol.done.astype(bool))
    assert np.array_equal(got["suicidal_mask"], ol.mask.astype(bool))
    losses = []
    for nb in range(K):
        ep_o, l_o = ol.step(nb)
        ep, loss = loop.step(nb)
        losses.append(loss)
        assert ep == ep_o and abs(loss - l_o) <= 1e-5 * abs(l_o), (nb, ep, ep_o, loss, l_o)
        assert np.float32(loop.eps) == ol.eps
    th = m.get_params().astype(np.float64)
    assert np.linalg.norm(th - ol.th) <= 1e-4 * np.linalg.norm(th - th0)
    tt = m.get_params(snk.SNK_NET_TARGET).astype(np.float64)
    assert np.linalg.norm(tt - ol.tt) <= 1e-4 * np.linalg.norm(tt - th0)   # synced after nb = 0 only
    for nb in range(K, 1000):
        _, loss = loop.step(nb)
        losses.append(loss)
    assert len(losses) == 1000 and np.all(np.isfinite(losses))
    e = np.float32(1.0)
    for _ in range(1000):
        e = max(np.float32(e - np.float32(1e-6)), np.float32(0.05))
    assert np.float32(loop.eps) == e and len(tr.buffer) == cap


def test_compute_D_episode_schedule_vs_oracle(snk):
    """compute_D.jl:33-142 at a small size (burn_in 5, thin 3, K 4, target
    rate 2, 10x10, 2 frames, capacity 300): fill, fresh RMSProp state, nb from
    1 with update_target_net! after nb = 2, 4, ...; snapshots before updates
    nb = 6, 9, 12, 15; Welford + centring. The device D follows the oracle
    replica (same decisions, own arithmetic) to 5e-3 of ||D|| (float drift
    over 14 RMSProp steps, whose g / sqrt(acc) amplifies tiny-gradient
    differences), while the replica on
    train!'s phase (nb from 0: syncs after nb = 0, 2, ...) misses by more than
    10x that: the test pins the phase. The Welford mean (~theta) within 5e-5."""
    from oracle_loops import OracleEpisodeLoop
    bs, C, cap, seed = 10, 2, 300, 0xD00D
    tr = snk.Trainer(n_envs=1, board_size=bs, n_frames=C, capacity=cap, target_update_rate=2, seed=seed)
    th0 = tr.model.get_params()
    lap = snk.compute_D(tr, K=4, thin=3, burn_in=5)
    D = lap.D()

    def replica(nb0):
        ol = OracleEpisodeLoop(bs, C, cap, seed, th0, rate=2)
        ol.fill()
        cols, nb = [], 1
        for pos in range(4):
            while nb < 6 + 3 * pos:
                ol.step(nb - 1 + nb0)
                nb += 1
            cols.append(ol.th.astype(np.float64))
        return oracle.welford_center(np.stack(cols))

    Dref, mref, _ = replica(1)
    err = np.linalg.norm(D - Dref) / np.linalg.norm(Dref)
    Dwrong, _, _ = replica(0)
    err_wrong = np.linalg.norm(D - Dwrong) / np.linalg.norm(Dwrong)
    print(f"compute_D: rel err {err:.2e} (train! phase: {err_wrong:.2e})")
    assert err <= 5e-3 and err_wrong > 10 * err
    assert np.linalg.norm(lap.mean() - mref) <= 5e-5 * np.linalg.norm(mref)


def test_compute_D_teacher_forced_vs_oracle(snk):
    """compute_D.jl:33-142 (episode schedule, nb from 1) teacher-forced, update
    by update: before every update nb the oracle replica takes the device's
    q_net, t_net and RMSProp state, plays the same episode (counter-RNG
    decisions; greedy ones from its own fp64 forward of the device q_net),
    draws the same batch and computes the loss and gradient. Per update:
    episode reward bit-exact, loss within rel 1e-5, gradient normwise 1e-5,
    (q_net, accumulator) after the update bit-exact with Float32 RMSProp of
    the device gradient, t_net == q_net exactly when nb % rate == 0 (else
    unchanged). The K = 6 snapshot columns are the device q_net before updates
    nb = 8, 12, ..., 28 bit for bit: the Welford mean/var and centred D equal
    the oracle's over those columns bit for bit. 10x10, 2 frames, capacity
    300, rate 3, epsilon 1 -> 0.4 (decay 0.025) so greedy decisions appear."""
    from oracle_loops import OracleEpisodeLoop
    bs, C, cap, seed, rate = 10, 2, 300, 0xD00D, 3
    K, thin, burn_in = 6, 4, 8
    tr = snk.Trainer(n_envs=1, board_size=bs, n_frames=C, capacity=cap, target_update_rate=rate, seed=seed,
                     epsilon=1.0, epsilon_end=0.4, decay=0.025, n_batches=1000)
    m = tr.model
    th0 = m.get_params()
    ol = OracleEpisodeLoop(bs, C, cap, seed, th0, rate=rate, epsilon=1.0, epsilon_end=0.4, decay=0.025)
    state = {"th": th0, "acc": np.zeros_like(th0), "tt": th0.copy(), "filled": False}
    after = {}                                   # nb -> device q_net after update nb

    def on_update(nb, loss):
        if not state["filled"]:                  # the device filled before update 1: follow it
            ol.fill()
            state["filled"] = True
        ol.th, ol.acc, ol.tt = state["th"].copy(), state["acc"].copy(), state["tt"].copy()
        ep_o, l_o = ol.step(nb)
        g = m.grad
        th, acc, tt = m.get_params(), m.get_params(snk.SNK_NET_OPT_STATE), m.get_params(snk.SNK_NET_TARGET)
        assert abs(loss - l_o) <= 1e-5 * abs(l_o), (nb, loss, l_o)
        assert np.linalg.norm(g - ol.last_grad) <= 1e-5 * np.linalg.norm(ol.last_grad), nb
        th_ref, acc_ref = oracle.rmsprop(state["th"], state["acc"], g)
        assert np.array_equal(th, th_ref) and np.array_equal(acc, acc_ref), nb
        assert np.array_equal(tt, th if nb % rate == 0 else state["tt"]), nb
        assert np.float32(tr.epsilon) == ol.eps, nb
        state.update(th=th, acc=acc, tt=tt)
        after[nb] = th

    lap = snk.compute_D(tr, K=K, thin=thin, burn_in=burn_in, on_update=on_update)
    snaps = [burn_in + thin * p for p in range(K)]
    assert sorted(after) == list(range(1, snaps[-1])), "updates nb = 1 .. 27 (none at the K-th snapshot)"
    cols = np.stack([after[nb - 1].astype(np.float64) for nb in snaps])
    Dref, mref, vref = oracle.welford_center(cols)
    assert np.array_equal(lap.D(), Dref) and np.array_equal(lap.mean(), mref) and np.array_equal(lap.var(), vref)
    assert ol.n_greedy > 0
    print(f"compute_D teacher-forced: {len(after)} updates, {ol.n_greedy} greedy oracle decisions")


def test_compute_D_stops_at_n_batches(snk):
    """compute_D.jl:58 `while nb <= n_batches`: when the K-th column would fall
    after n_batches, the loop runs updates 1..n_batches and returns nothing."""
    tr = snk.Trainer(n_envs=1, board_size=10, n_frames=2, capacity=200, seed=3, n_batches=9)
    losses = []
    with pytest.warns(RuntimeWarning, match="before the K-th snapshot"):
        out = snk.compute_D(tr, K=3, thin=2, burn_in=6, on_update=lambda nb, loss: losses.append(nb))
    assert out is None and losses == list(range(1, 10))
    tr = snk.Trainer(n_envs=1, board_size=10, n_frames=2, capacity=200, seed=3, n_batches=9)
    with pytest.raises(ValueError, match="n_batches to >= 10"):
        snk.compute_D(tr, K=3, thin=2, burn_in=6, strict=True)
