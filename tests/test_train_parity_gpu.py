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
