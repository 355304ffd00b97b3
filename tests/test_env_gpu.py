"""GPU parity of the batched env kernel against the oracle (bit-exact integer
state) and against the reference's GIF trajectories."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _gif_replay(snk, fx, n_frames):
    g = snk.SnakeGame(10, n_frames, n_envs=1, autoreset=False)
    boards = fx["boards_cells"]
    first = n_frames
    ep = None
    for t, a in enumerate(fx["act_idx"]):
        snk.step_(g, [int(a)])
        assert np.array_equal(g.board_cells()[0], boards[first + t]), f"step {t + 1}"
        o = g.last()
        ep = o["ep_reward"][0]
    return g, ep


def test_gif_double3_on_device(snk, golden):
    g, ep = _gif_replay(snk, golden["double3"], 2)
    assert g.score[0] == 33 and g.lost[0]
    assert ep == np.float32(29.969957)
    assert g.check_faults() == 0


def test_gif_vanilla_on_device(snk, golden):
    g, _ = _gif_replay(snk, golden["vanilla1"], 1)
    assert g.score[0] == 8 and not g.lost[0]


def test_gif_double3_absolute_directions(snk, golden):
    """step!(game, CartesianIndex) with absolute directions (utils.jl:100)."""
    fx = golden["double3"]
    g = snk.SnakeGame(10, 2, n_envs=1)
    for t, d in enumerate(fx["dirs"]):
        snk.step_(g, snk.ALL_ACTIONS[int(d)])
    assert np.array_equal(g.board_cells()[0], fx["boards_cells"][-1])
    assert g.score[0] == 33


@pytest.mark.parametrize("bs,C", [(10, 2), (12, 2), (12, 1), (20, 2)])
def test_random_actions_bitexact_vs_oracle(snk, bs, C):
    """Counter-RNG actions, auto-reset, 520 lockstep steps (past the 500-step
    truncation of utils.jl:88): every output and every board bit-exact."""
    n, T, seed = 192, 520, 0x5EED + bs
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    ob = oracle.OracleBatch(n, bs, C)
    act = snk.DeviceArray(n, np.uint8)
    saw_done = saw_trunc = 0
    for t in range(T):
        snk.synth_actions_dev(g, seed, act)
        a = act.numpy()
        assert np.array_equal(a, oracle.synth_actions(seed, n, t))
        snk.step_indices_dev(g, act.ptr)
        ref = ob.step(a, want_frames=False)
        o = g.last()
        assert np.array_equal(o["reward"], ref["reward"]), t
        assert np.array_equal(o["done"], ref["done"]), t
        m = ref["mask"][:, 0] | (ref["mask"][:, 1] << 1) | (ref["mask"][:, 2] << 2)
        assert np.array_equal(o["mask"], m), t
        dirs = ref["prev_dir"] | (ref["dir"] << 2) | (ref["done"] << 4)
        assert np.array_equal(o["dirs"], dirs), t
        if t % 37 == 0 or t == T - 1:
            assert np.array_equal(g.board_cells(), ob.boards()), t
        saw_done += int(ref["done"].sum())
    assert saw_done > 0
    sc = ob.scalars()
    gs = g._scalars()
    assert np.array_equal(gs["score"], sc["score"]) and np.array_equal(gs["len"], sc["len"])
    assert np.array_equal(gs["steps"], sc["steps"])
    assert np.array_equal(gs["episode_reward"], sc["episode_reward"])
    assert g.check_faults() == 0


def test_truncation_at_500_steps(snk):
    """A snake circling forever is lost at real step 500 (utils.jl:88) and the
    virtual step flags every action suicidal from step 499 (n_frames = 2)."""
    g = snk.SnakeGame(10, 2, n_envs=1)
    ob = oracle.OracleBatch(1, 10, 2)
    # circle in a 2x2 loop: U, R, D, L ... as absolute directions
    loop = [snk.U, snk.R, snk.D, snk.L]
    for k in range(500):
        d = loop[k % 4]
        snk.step_(g, d)
        a_idx = snk.available_action_codes(ob.scalars()["prev_dir"][0]).index(snk.ALL_ACTIONS.index(d))
        ref = ob.step(np.array([a_idx], np.uint8), want_frames=False)
        o = g.last()
        assert o["done"][0] == ref["done"][0] and o["mask"][0] == (ref["mask"][0] @ [1, 2, 4])
        if k == 498:
            assert o["mask"][0] == 7 and not o["done"][0]
    assert g.lost[0] and o["reward"][0] == np.float32(-1)


def test_step_store_replay_frames(snk):
    """Fused step + store!: each replay slot holds b_{t-C}..b_t exactly as the
    oracle's frames (utils.jl:141-149) and the metadata of the transition."""
    n, T, bs, C, seed = 128, 40, 12, 2, 99
    g = snk.SnakeGame(bs, C, n_envs=n, autoreset=True)
    rb = snk.ReplayBuffer(n * T, board_size=bs, n_frames=C, batch_size=64)
    ob = oracle.OracleBatch(n, bs, C)
    act = snk.DeviceArray(n, np.uint8)
    ref_frames, ref_meta = [], []
    for t in range(T):
        snk.synth_actions_dev(g, seed, act)
        snk.step_indices_dev(g, act.ptr, replay=rb)
        r = ob.step(act.numpy())
        ref_frames.append(r["frames"])
        ref_meta.append(r)
    assert len(rb) == n * T
    idx = np.arange(n * T, dtype=np.int64)
    got = snk.stack_exp(rb, idx)
    frames = np.concatenate(ref_frames)           # [T*n, C+1, bs*bs]
    assert np.array_equal(got["states"], frames[:, :C].astype(np.float32))
    assert np.array_equal(got["next_states"], frames[:, 1:].astype(np.float32))
    rew = np.concatenate([m["reward"] for m in ref_meta])
    done = np.concatenate([m["done"] for m in ref_meta])
    mask = np.concatenate([m["mask"] for m in ref_meta])
    assert np.array_equal(got["rewards"], rew)
    assert np.array_equal(got["dones"], done.astype(bool))
    assert np.array_equal(got["suicidal_mask"], mask.astype(bool))
    act_all = np.concatenate([oracle.synth_actions(seed, n, t) for t in range(T)])
    assert np.array_equal(got["actions"], act_all.astype(np.int32) + 1)   # 1-based (utils.jl:363)


def test_replay_ring_wrap_and_sample(snk):
    bs, C = 10, 2
    rb = snk.ReplayBuffer(100, board_size=bs, n_frames=C, batch_size=64)
    assert len(rb) == 0 and rb.position == 1
    B = 30
    for k in range(5):   # 150 stores into capacity 100 -> wraps
        fr = np.full((B, C + 1, bs * bs), k, np.int8)
        snk.store_(rb, fr, np.zeros(B), np.full(B, k, np.float32), np.zeros(B), np.zeros((B, 3)),
                   np.zeros(B))
    assert len(rb) == 100 and rb.count == 150 and rb.position == 51
    got = snk.stack_exp(rb, np.arange(100))
    # slots 0..49 were overwritten by stores 100..149 (k = 3, 4), 50..99 hold k = 1, 2
    expect = np.array([3] * 20 + [4] * 30 + [1] * 10 + [2] * 30 + [3] * 10, np.float32)
    assert np.array_equal(got["rewards"], expect)
    idx, Bs = snk.sample(rb, seed=7, draw=0)
    ids = idx.numpy()[:Bs]
    assert Bs == 64 and len(set(ids.tolist())) == 64 and ids.min() >= 0 and ids.max() < 100
    idx2, _ = snk.sample(rb, seed=7, draw=1)
    assert not np.array_equal(idx2.numpy(), ids)


def _floyd_ref(seed, draw, n_len, batch):
    """Floyd's algorithm with the device's counter RNG (snk_common.hpp rng_hash)."""
    M = (1 << 64) - 1

    def sm(x):
        z = (x + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    B = min(batch, n_len)
    chosen, out = set(), []
    for n in range(B):
        h = sm(sm(seed ^ ((draw * 0xD1B54A32D192ED03) & M)) ^ n)
        t = (h * (n_len - B + n + 1)) >> 64
        v = n_len - B + n if t in chosen else t
        chosen.add(v)
        out.append(v)
    return out


@pytest.mark.parametrize("batch", [64, 17, 100])
def test_sample_matches_floyd_reference(snk, batch):
    """The wave-ballot sampler (batch <= 64) and the LDS-set sampler draw the
    exact subset Floyd's algorithm gives for the same counter RNG."""
    bs, C = 10, 2
    rb = snk.ReplayBuffer(200, board_size=bs, n_frames=C, batch_size=batch)
    for k in range(5):
        fr = np.zeros((30, C + 1, bs * bs), np.int8)
        snk.store_(rb, fr, np.zeros(30), np.zeros(30, np.float32), np.zeros(30), np.zeros((30, 3)), np.zeros(30))
    for draw in range(4):
        idx, B = snk.sample(rb, seed=11, draw=draw)
        assert idx.numpy()[:B].tolist() == _floyd_ref(11, draw, 150, batch)
