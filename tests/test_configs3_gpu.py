"""BASELINE.json configs[3] at its own per-rank size, on one GPU, and the
configs[1] bench graph (4096 envs) with greedy actions.

configs[3] is 262,144 lockstep envs sharded over 8 MI355X: each rank runs
32,768 envs of 12x12 (2 frames) with its own 50k replay shard and B = 64 per
update (the ranks' gradients are then mean-all-reduced; that exchange is
covered by tests/test_dist_*.py). This file runs ONE rank's shard exactly as
bench.py --workload configs3 times it: Trainer(32,768 envs, capacity 50,000,
B = 64, graph_unroll 8), and replays it on the oracle (utils.jl:389-482,
train!/fill_buffer!) decision by decision.

epsilon is 0.25, so three quarters of the actions are greedy: they come from
conv_h3f_kernel's act forward (an 8,193-workgroup grid at 32,768 states),
whose h3 weight scale inside a captured graph comes from the previous
iteration's grad_update (the chained weight-max partials, snk_trainer.hip) for
iterations 1..7, from a rescan for iteration 0. The trainer's act trace
(snk_trainer_set_act_trace) makes each iteration's actions and Q values
inside the graph observable; the gradient trace (snk_trainer_set_trace) each
update's gradient.

The same replay runs at 4096 envs with the bench's own epsilon 0.05
(bench.py's workload: 95 % of the actions greedy from conv_h3f_kernel +
dense_h3_kernel, whose per-sample a3 scale is reduced in conv_h3f's epilogue:
the round-4 regression class), 1,024 sampled states per
iteration (every fourth env, all four workgroup slots over the iterations).

Tolerances:
  env outputs, boards, replay ring (all 50,000 slots)       bit-exact
  explored actions (counter stream)                          bit-exact
  greedy actions vs the device's own Q (first argmax)        exact
  Q of >= 2,048 sampled states, every iteration and every
    workgroup slot class, vs the fp64 oracle at that
    iteration's parameters                                   |q - q_ref| <= 1e-5 max(1, |q_ref|)
  greedy actions vs the oracle's first argmax (top-2 margin > 1e-4)   exact
  chained-scale Q (iterations 1..7) vs a fresh forward of the same
    weights and states (weight max rescanned)                bit-exact
  8 teacher-forced updates: loss rel 1e-5, gradient normwise
    1e-5 (kink-aware, tests/kinks.py); q_net, accumulator,
    t_net after the graph == Float32 RMSProp of the traced
    gradients                                                bit-exact
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle
from devrng import TRAINER_SAMPLE_SALT, explore_np, first_argmax_np, floyd
from kinks import grad_parity

pytestmark = pytest.mark.gpu


def _oracle_q(bs, C, params, x, workers=16):
    """oracle.qnet_forward over many states, split across threads (the C call
    releases the GIL)."""
    parts = np.array_split(np.arange(len(x)), min(workers, len(x)))
    with ThreadPoolExecutor(len(parts)) as ex:
        out = list(ex.map(lambda ix: oracle.qnet_forward(bs, C, params, x[ix]), parts))
    return np.concatenate(out)


def _sample_envs(n, it, k=256):
    """k envs spread over the whole grid (one every n/k, i.e. every 32nd
    workgroup of four), each iteration shifted so the four slot positions of
    a workgroup and every workgroup residue are all visited."""
    step = n // k
    return np.arange(k) * step + (it * 37 + np.arange(k) * 5) % step


@pytest.mark.parametrize("n,eps,k", [(32768, 0.25, 256), (4096, 0.05, 1024)], ids=["configs3_shard", "configs1_eps005"])
def test_configs3_per_rank_shard_trajectory_vs_oracle(snk, n, eps, k):
    bs, C, cap, B, rate, U, seed = 12, 2, 50_000, 64, 5, 8, 0xC3C3 ^ n
    eps = np.float32(eps)
    tr = snk.Trainer(n_envs=n, board_size=bs, n_frames=C, capacity=cap, batch_size=B, n_batches=10_000,
                     target_update_rate=rate, epsilon=float(eps), epsilon_end=float(eps), decay=0.0, seed=seed,
                     graph_unroll=U)
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
    st = {"count": 0, "t": 0, "q_checked": 0, "greedy_vs_oracle": 0}
    worst = {"q": 0.0}

    def check_acts(a, q, th, it):
        """One iteration's actions and act-forward Q (device trace slot) against
        the counter stream, the device's own argmax and the oracle at th."""
        states = ob.states()
        ex = explore_np(seed, n, st["t"], eps)
        rnd = ex >= 0
        assert np.array_equal(a[rnd], ex[rnd]), (st["t"], "explored actions")
        assert abs(rnd.mean() - eps) < 0.05 and (~rnd).sum() > 0.7 * n
        assert np.array_equal(a[~rnd], first_argmax_np(q[~rnd])), (st["t"], "greedy action != argmax of device Q")
        sel = _sample_envs(n, it, k)
        qref = _oracle_q(bs, C, th, states[sel].astype(np.float32))
        err = np.abs(q[sel] - qref) / np.maximum(1.0, np.abs(qref))
        worst["q"] = max(worst["q"], float(err.max()))
        assert err.max() <= 1e-5, (st["t"], float(err.max()), int(sel[np.argmax(err.max(1))]))
        st["q_checked"] += len(sel)
        g = sel[~rnd[sel]]
        top = np.sort(qref[~rnd[sel]], axis=1)
        ok = top[:, 2] - top[:, 1] > 1e-4
        assert np.array_equal(a[g][ok], first_argmax_np(qref[~rnd[sel]])[ok]), st["t"]
        st["greedy_vs_oracle"] += int(ok.sum())
        return states

    def oracle_step(a):
        out = ob.step(a)
        k = (st["count"] + np.arange(n)) % cap
        frames[k], o_act[k], o_rew[k], o_done[k], o_mask[k] = out["frames"], a, out["reward"], out["done"], out["mask"]
        st["count"] += n
        st["t"] += 1
        return out

    def check_env(out):
        o = tr.game.last("reward", "done", "mask")
        assert np.array_equal(o["reward"], out["reward"]) and np.array_equal(o["done"], out["done"]), st["t"]
        assert np.array_equal(o["mask"], out["mask"] @ np.array([1, 2, 4], np.uint8)), st["t"]
        assert np.array_equal(tr.game.board_cells(), ob.boards()), st["t"]

    # fill_buffer! (utils.jl:389-402): more than 50,000 transitions = 2 lockstep steps of
    # 32,768 envs (13 of 4096), one single-iteration graph each (trace slot 0), greedy
    # actions from theta_0
    th0 = m.get_params()
    nfill = cap // n + 1
    for it in range(nfill):
        tr.run(1, learn=False, graph=True)
        a, q = aring.numpy()[0], qring.numpy()[0]
        check_acts(a, q, th0, it)
        out = oracle_step(a)
        check_env(out)
    assert len(tr.buffer) == cap and st["count"] == nfill * n

    # ONE replay of the captured 8-iteration graph: act forward (conv_h3f_kernel, 32,768
    # states) + step/store + one B = 64 update per iteration
    th, acc, tt = m.get_params(), m.get_params(snk.SNK_NET_OPT_STATE), m.get_params(snk.SNK_NET_TARGET)
    tr.run(U, learn=True, graph=True)
    acts, qs = aring.numpy(), qring.numpy()
    gdev = np.empty((U, P), np.float32)
    gdev[:, perm] = gring.numpy()
    losses = tr.losses
    sseed = seed ^ TRAINER_SAMPLE_SALT
    keep_end = [(w, m.get_params(w)) for w in (snk.SNK_NET_Q, snk.SNK_NET_TARGET, snk.SNK_NET_OPT_STATE)]

    def restore():
        def put():
            for w, v in keep_end:
                m.set_params(v, w)
        return put

    worst_loss = worst_grad = 0.0
    kinks = 0
    th_it, states_it = [], []
    for i in range(U):
        th_it.append(th)
        states_it.append(check_acts(acts[i], qs[i], th, nfill + i))
        out = oracle_step(acts[i])
        ids = floyd(sseed, i, min(st["count"], cap), B)
        f = frames[ids].copy()
        batch = (f, o_act[ids].copy(), o_rew[ids].copy(), o_done[ids].copy(), o_mask[ids].copy())
        ref = oracle.dqn_loss_grad_kinks(bs, C, th, tt, f[:, :C], batch[1], batch[2], f[:, 1:], batch[3], batch[4])
        rl = abs(losses[i] - ref[0]) / abs(ref[0])
        assert rl <= 1e-5, (i, losses[i], ref[0])
        rg, rk, nk = grad_parity(snk, m, bs, C, th, tt, batch, gdev[i], restore=restore, ref=ref)
        worst_loss, worst_grad, kinks = max(worst_loss, rl), max(worst_grad, rk), kinks + nk
        th, acc = oracle.rmsprop(th, acc, gdev[i])
        if i % rate == 0:
            tt = th.copy()
    check_env(out)
    assert np.array_equal(keep_end[0][1], th) and np.array_equal(keep_end[2][1], acc)
    assert np.array_equal(keep_end[1][1], tt)
    s = tr.stats()
    assert s["updates"] == U and s["nb"] == U and s["env_steps"] == st["t"] * n

    # the replay ring: every one of the 50,000 slots (it wrapped 6 times at 32,768 envs)
    got = snk.stack_exp(tr.buffer, np.arange(cap))
    assert np.array_equal(got["states"], frames[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], frames[:, 1:].astype(np.float32))
    assert np.array_equal(got["actions"], o_act + 1) and np.array_equal(got["rewards"], o_rew)
    assert np.array_equal(got["dones"], o_done.astype(bool))
    assert np.array_equal(got["suicidal_mask"], o_mask.astype(bool))

    # the chained weight scale: iterations 1..7's act forwards (weight-max partials written by
    # the previous update's grad_update) against a fresh forward of the same weights and
    # states, which rescans the weight image; iteration 0 (rescanned inside the graph) is
    # the control
    for i in range(U):
        m.set_params(th_it[i])
        qf = m.forward(states_it[i].astype(np.float32))
        assert np.array_equal(qf, qs[i]), (i, float(np.abs(qf - qs[i]).max()))
    print(f"{n} envs, eps {eps}: {st['t']} lockstep steps of {n} envs, {st['q_checked']} Q values vs the oracle "
          f"(max err {worst['q']:.2e}), {st['greedy_vs_oracle']} greedy actions vs the oracle argmax; "
          f"{U} updates: loss rel max {worst_loss:.2e}, gradient max {worst_grad:.2e} ({kinks} kink decision(s))")
