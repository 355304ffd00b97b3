"""Composed-loop parity: the device train! loops replayed on the CPU oracle,
decision by decision (utils.jl:389-482 train!/fill_buffer!, compute_D.jl:89-138).

Actions and replay draws come from the device's counter RNG, restated in
tests/devrng.py; everything else (env, replay contents, TD target, Huber,
gradient, RMSProp, target sync, epsilon decay) is checked against the oracle.

Tolerances:
  env state, replay contents, actions       bit-exact
  per-update loss (teacher-forced)          relative 1e-5
  per-update gradient (teacher-forced)      normwise 1e-5
  RMSProp step given the device gradient    bit-exact
  free-running theta after all updates      ||th_dev - th_orc|| <= 1e-3 ||th_dev - th_0||
"""
import numpy as np
import pytest

import oracle
from devrng import TRAINER_SAMPLE_SALT, explore, first_argmax, floyd
from kinks import grad_parity

pytestmark = pytest.mark.gpu


class OracleReplay:
    """store! / stack_exp on the CPU: ring of (b_{t-C}..b_t, action, reward, done, mask)."""

    def __init__(self, cap, C, nc):
        self.cap, self.count = cap, 0
        self.frames = np.zeros((cap, C + 1, nc), np.int8)
        self.act = np.zeros(cap, np.int32)
        self.rew = np.zeros(cap, np.float32)
        self.done = np.zeros(cap, np.uint8)
        self.mask = np.zeros((cap, 3), np.uint8)

    def store(self, step_out, act):
        for e in range(len(act)):
            k = self.count % self.cap
            self.frames[k] = step_out["frames"][e]
            self.act[k] = act[e]
            self.rew[k] = step_out["reward"][e]
            self.done[k] = step_out["done"][e]
            self.mask[k] = step_out["mask"][e]
            self.count += 1

    def __len__(self):
        return min(self.count, self.cap)

    def loss_grad(self, bs, C, qp, tp, ids):
        fr = self.frames[ids]
        return oracle.dqn_loss_grad(bs, C, qp, tp, fr[:, :C], self.act[ids], self.rew[ids], fr[:, 1:],
                                    self.done[ids], self.mask[ids])


def _acts_ok(acts, seed, t, eps, qp, bs, C, states):
    """Every env's action equals the restated epsilon_greedy; greedy ones the
    oracle's first argmax (ties within 1e-4 skipped). Returns #greedy checked."""
    greedy = [e for e in range(len(acts)) if explore(seed, e, t, eps) is None]
    for e in range(len(acts)):
        r = explore(seed, e, t, eps)
        if r is not None:
            assert acts[e] == r, (t, e)
    if greedy:
        q = oracle.qnet_forward(bs, C, qp, states[greedy].astype(np.float32))
        for e, qe in zip(greedy, q):
            top = np.sort(qe)
            if top[2] - top[1] > 1e-4:
                assert acts[e] == first_argmax(qe), (t, e, qe)
    return len(greedy)


def test_lockstep_trainer_trajectory_vs_oracle(snk):
    """The graph-replayed lockstep trainer (snk_trainer_run) for 13 fill
    iterations and 12 updates at 16 envs of 10x10, 2 frames, B = 32, target
    sync every 4 updates, epsilon 0.6 -> 0.5 decaying 0.01 per update:
    every iteration's actions, env outputs and boards, every replay slot, every
    update's batch, loss and gradient, RMSProp step, target sync and epsilon
    agree with the oracle; the free-running oracle trajectory ends within
    1e-3 of the device's parameter change."""
    bs, C, n, cap, B, rate, seed = 10, 2, 16, 200, 32, 4, 0xC0FFEE
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=cap, batch_size=B, n_batches=11,
                     target_update_rate=rate, epsilon=0.6, epsilon_end=0.5, decay=0.01, seed=seed)
    m = tr.model
    from snake_amd import _lib
    act_ptr = _lib.vp()
    _lib.call("snk_trainer_act_ptr", tr.handle, _lib.C.byref(act_ptr))
    ob = oracle.OracleBatch(n, bs, C)
    orb = OracleReplay(cap, C, bs * bs)
    th0 = m.get_params()
    th_o, acc_o, tt_o = th0.copy(), np.zeros_like(th0), th0.copy()     # free-running oracle
    eps = np.float32(0.6)
    sseed = seed ^ TRAINER_SAMPLE_SALT
    t, n_greedy = 0, 0

    def one_iteration(learn):
        nonlocal t, n_greedy
        qp = m.get_params()
        states = ob.states()
        assert np.array_equal(snk.assemble_state_(tr.game).astype(np.int8), states)
        tr.run(1, learn=learn, graph=True)
        a = np.zeros(n, np.uint8)
        _lib.call("snk_memcpy_d2h", a.ctypes.data_as(_lib.vp), act_ptr, n)
        n_greedy += _acts_ok(a, seed, t, eps, qp, bs, C, states)
        out = ob.step(a)
        o = tr.game.last("reward", "done", "mask")
        assert np.array_equal(o["reward"], out["reward"]) and np.array_equal(o["done"], out["done"])
        assert np.array_equal(o["mask"], out["mask"] @ np.array([1, 2, 4], np.uint8))
        orb.store(out, a)
        t += 1
        return qp

    # fill_buffer!: more than cap transitions, one iteration at a time
    while orb.count <= cap:
        one_iteration(False)
    assert len(tr.buffer) == len(orb) == cap
    got = snk.stack_exp(tr.buffer, np.arange(cap))
    assert np.array_equal(got["states"], orb.frames[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], orb.frames[:, 1:].astype(np.float32))
    assert np.array_equal(got["actions"], orb.act + 1) and np.array_equal(got["rewards"], orb.rew)
    assert np.array_equal(got["suicidal_mask"], orb.mask.astype(bool))

    for u in range(12):
        acc = m.get_params(snk.SNK_NET_OPT_STATE)
        tp = m.get_params(snk.SNK_NET_TARGET)
        qp = one_iteration(True)
        ids = floyd(sseed, u, len(orb), B)
        lref, gref, _ = orb.loss_grad(bs, C, qp, tp, ids)
        loss = tr.losses[u]
        assert abs(loss - lref) <= 1e-5 * abs(lref), (u, loss, lref)
        g = m.grad
        assert np.linalg.norm(g - gref) <= 1e-5 * np.linalg.norm(gref), u
        th_ref, acc_ref = oracle.rmsprop(qp, acc, g)
        th = m.get_params()
        assert np.array_equal(th, th_ref) and np.array_equal(m.get_params(snk.SNK_NET_OPT_STATE), acc_ref), u
        assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), th if u % rate == 0 else tp), u
        eps = max(np.float32(eps - np.float32(0.01)), np.float32(0.5))
        assert np.float32(tr.stats()["epsilon"]) == eps
        # the oracle on its own trajectory (same transitions and draws)
        _, go, _ = orb.loss_grad(bs, C, th_o, tt_o, ids)
        th_o, acc_o = oracle.rmsprop(th_o, acc_o, go.astype(np.float32))
        if u % rate == 0:
            tt_o = th_o.copy()
    st = tr.stats()
    assert st["updates"] == 12 and st["nb"] == 12 and st["env_steps"] == t * n
    assert n_greedy > 0
    th = m.get_params()
    drift = np.linalg.norm(th.astype(np.float64) - th_o) / np.linalg.norm(th.astype(np.float64) - th0)
    print(f"free-running drift {drift:.3e} after 12 updates; {n_greedy} greedy actions checked")
    assert drift <= 1e-3


def test_trainer_nb_phase_and_partial_iteration(snk):
    """set_nb(1) puts update_target_net! on the compute_D.jl phase (nb = rate,
    2 rate, ...; never on the first update), and train_ with
    updates_per_iter = 3 runs exactly n_batches + 1 = 8 updates (2 full
    iterations + one partial of 2)."""
    tr = snk.Trainer(n_envs=32, board_size=10, n_frames=2, capacity=100, batch_size=16, n_batches=7,
                     target_update_rate=3, updates_per_iter=3, seed=5)
    snk.fill_buffer_(tr)
    m = tr.model
    tr.set_nb(1)
    t0 = m.get_params(snk.SNK_NET_TARGET)
    tr.run(1)                          # nb = 1, 2, 3: synced after nb = 3 only
    assert not np.array_equal(m.get_params(snk.SNK_NET_TARGET), t0)
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), m.get_params())
    tr.set_nb(1)
    t1 = m.get_params(snk.SNK_NET_TARGET)
    tr.run_partial(2)                  # nb = 1, 2: no sync
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), t1)
    tr2 = snk.Trainer(n_envs=32, board_size=10, n_frames=2, capacity=100, batch_size=16, n_batches=7,
                      target_update_rate=3, updates_per_iter=3, seed=5)
    st = snk.train_(tr2)
    assert st["updates"] == 8 and len(tr2.losses) == 8


def test_trainer_graph_survives_workspace_growth(snk):
    """A model call with a batch larger than the trainer's envs reallocates the
    shared act workspace; the next trainer run re-captures its graphs instead
    of replaying freed pointers, and matches an untouched twin run."""
    outs = []
    for grow in (False, True):
        tr = snk.Trainer(n_envs=64, board_size=10, n_frames=2, capacity=300, batch_size=16, n_batches=0, seed=9)
        snk.fill_buffer_(tr)
        tr.run(2)
        if grow:
            x = np.zeros((1500, 2, 100), np.float32)
            tr.model.forward(x)                       # grows the act workspace past 64 samples
            g2 = snk.SnakeGame(10, 2, n_envs=700, autoreset=True)
            snk.epsilon_greedy(g2, tr.model, 0.1)     # and the env-forward one
        tr.run(3)
        outs.append((tr.model.get_params(), tr.losses))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_bench_graph_trajectory_vs_oracle(snk):
    """The graph bench.py times, replayed on the oracle update by update
    (utils.jl:434-482): 4096 lockstep 12x12 games, 2 frames, B = 64, capacity
    50,000, graph_unroll 8, so each snk_trainer_run(8) is ONE captured graph of
    8 iterations of conv_h3f_kernel act forward (>= 1024 states) + the
    wmax_scan sample rider, env_step_kernel with store!, upd_fwd_kernel<12,2>
    update forward, the backward kernels and grad_update_kernel. epsilon 1 (no
    decay) in the checked window, so every action is the restated counter
    stream (the 4096-state greedy forward is test_configs1_act_forward_4096_vs_oracle).
    Target sync every 5 updates (nb = 0, 5, 10, 15) to put syncs inside graphs.
    The trainer's gradient trace (snk_trainer_set_trace: one device copy of
    each update's finished gradient, appended to the same graph) makes the
    8 updates inside a graph observable.

    After the fill (13 iterations) and after each of 2 graphs (16 updates,
    the replay ring wrapping past 50,000):
      boards, the last iteration's outputs and actions          bit-exact
      replay ring (all 50,000 slots) at the end                 bit-exact
      every update, teacher-forced: the oracle takes the device's q_net,
        t_net and accumulator before the update (start of the graph,
        then RMSProp of the traced device gradients) and the Floyd draw
          loss (tr.losses)                                      relative 1e-5
          gradient                                              normwise 1e-5, kink-aware
            (tests/kinks.py: a relu decision at z within fp32 rounding of 0 may go
            either way; such an update is re-run on the device, and the oracle under
            the device's decisions must then agree, every differing decision at a kink)
      q_net, accumulator, t_net after each graph == Float32 RMSProp of the
        8 traced gradients from the graph-start state, t_net synced after
        nb % 5 == 0                                             bit-exact
    """
    from devrng import rng_hash
    bs, C, n, cap, B, rate, seed, U = 12, 2, 4096, 50_000, 64, 5, 0xBE4C, 8
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=cap, batch_size=B, n_batches=10_000,
                     target_update_rate=rate, epsilon=1.0, epsilon_end=1.0, decay=0.0, seed=seed, graph_unroll=U)
    m = tr.model
    P = m.P
    perm = m.flux_index()
    ring = snk.DeviceArray((U, P), np.float32)
    from snake_amd import _lib
    act_ptr = _lib.vp()
    _lib.call("snk_trainer_act_ptr", tr.handle, _lib.C.byref(act_ptr))
    ob = oracle.OracleBatch(n, bs, C)
    nc = bs * bs
    frames = np.zeros((cap, C + 1, nc), np.int8)
    o_act = np.zeros(cap, np.int32)
    o_rew = np.zeros(cap, np.float32)
    o_done = np.zeros(cap, np.uint8)
    o_mask = np.zeros((cap, 3), np.uint8)
    count, t = 0, 0
    sseed = seed ^ TRAINER_SAMPLE_SALT
    salt = seed ^ 0xA5A5A5A5A5A5A5A5

    def oracle_iteration():
        nonlocal count, t
        a = np.array([(rng_hash(salt, e, t) >> 32) % 3 for e in range(n)], np.uint8)   # explore() at eps = 1
        out = ob.step(a)
        k = (count + np.arange(n)) % cap
        frames[k], o_act[k], o_rew[k], o_done[k], o_mask[k] = out["frames"], a, out["reward"], out["done"], out["mask"]
        count += n
        t += 1
        return a, out

    def check_env(a, out):
        got = np.zeros(n, np.uint8)
        _lib.call("snk_memcpy_d2h", got.ctypes.data_as(_lib.vp), act_ptr, n)
        assert np.array_equal(got, a), t
        o = tr.game.last("reward", "done", "mask")
        assert np.array_equal(o["reward"], out["reward"]) and np.array_equal(o["done"], out["done"]), t
        assert np.array_equal(o["mask"], out["mask"] @ np.array([1, 2, 4], np.uint8)), t
        assert np.array_equal(tr.game.board_cells(), ob.boards()), t

    snk.fill_buffer_(tr)                                   # 13 iterations: one 8-graph + 5 single graphs
    for _ in range(13):
        a, out = oracle_iteration()
    check_env(a, out)
    assert len(tr.buffer) == cap and count == 13 * n

    tr.set_trace(ring)
    u = 0
    worst_loss = worst_grad = 0.0
    kinks = 0

    def save_state():                                      # the graph-end state, restored after a kink replay
        keep = [(w, m.get_params(w)) for w in (snk.SNK_NET_Q, snk.SNK_NET_TARGET, snk.SNK_NET_OPT_STATE)]

        def put():
            for w, v in keep:
                m.set_params(v, w)
        return put

    for graph in range(2):
        th = m.get_params()
        acc = m.get_params(snk.SNK_NET_OPT_STATE)
        tt = m.get_params(snk.SNK_NET_TARGET)
        draws = []
        for _ in range(U):
            a, out = oracle_iteration()
            f_ids = floyd(sseed, u + len(draws), min(count, cap), B)
            draws.append((f_ids, frames[f_ids].copy(), o_act[f_ids].copy(), o_rew[f_ids].copy(),
                          o_done[f_ids].copy(), o_mask[f_ids].copy()))
        tr.run(U, learn=True, graph=True)                 # ONE replay of the captured 8-iteration graph
        check_env(a, out)
        losses = tr.losses[u:u + U]
        gdev = np.empty((U, P), np.float32)
        gdev[:, perm] = ring.numpy()
        for k, (ids, f, ac, rw, dn, mk) in enumerate(draws):
            ref = oracle.dqn_loss_grad_kinks(bs, C, th, tt, f[:, :C], ac, rw, f[:, 1:], dn, mk)
            rl = abs(losses[k] - ref[0]) / abs(ref[0])
            assert rl <= 1e-5, (u, losses[k], ref[0])
            rg, rk, nk = grad_parity(snk, m, bs, C, th, tt, (f, ac, rw, dn, mk), gdev[k], restore=save_state,
                                     ref=ref)
            worst_loss, worst_grad = max(worst_loss, rl), max(worst_grad, rk)
            kinks += nk
            if nk:
                print(f"update {u}: gradient {rg:.2e} vs the oracle's relu decisions, {rk:.2e} under the device's "
                      f"({nk} kink decision(s))")
            th, acc = oracle.rmsprop(th, acc, gdev[k])
            if u % rate == 0:
                tt = th.copy()
            u += 1
        assert np.array_equal(m.get_params(), th), graph
        assert np.array_equal(m.get_params(snk.SNK_NET_OPT_STATE), acc), graph
        assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), tt), graph
    assert np.array_equal(m.get_params(snk.SNK_NET_TARGET), m.get_params())   # nb = 15 synced last
    st = tr.stats()
    assert st["updates"] == 16 and st["nb"] == 16 and st["env_steps"] == t * n
    got = snk.stack_exp(tr.buffer, np.arange(cap))
    assert np.array_equal(got["states"], frames[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], frames[:, 1:].astype(np.float32))
    assert np.array_equal(got["actions"], o_act + 1) and np.array_equal(got["rewards"], o_rew)
    assert np.array_equal(got["dones"], o_done.astype(bool))
    assert np.array_equal(got["suicidal_mask"], o_mask.astype(bool))
    print(f"bench graph, 16 teacher-forced updates: loss rel max {worst_loss:.2e}, gradient max {worst_grad:.2e} "
          f"({kinks} relu kink decision(s) accounted)")
