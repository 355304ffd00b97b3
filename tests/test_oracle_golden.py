"""CPU: the oracle restatement is pinned against the reference's own artefacts
(SURVEY.md §8c): the BSON trainer's food list and Xoshiro state, both
best-game GIFs frame by frame, and the BSON Q-net's greedy actions."""
import numpy as np

import oracle


def test_food_list_matches_bson(golden):
    fx = golden["bson"]
    cells, st = oracle.food_list(10, 42, 50)
    got = [[int(c) % 10 + 1, int(c) // 10 + 1] for c in cells]
    assert got == fx["food_list_1based"]
    # RNG state after the 100 draws of structs.jl:70 equals the stored food_rng
    assert ["%016x" % int(w) for w in st] == fx["food_rng_state_s0_s4_hex"][:4]
    s0 = oracle.xoshiro_seed(42)
    assert "%016x" % int(s0[4]) == fx["food_rng_state_s0_s4_hex"][4]   # s4 = s0+3s1+5s2+7s3


def test_bson_board_shows_wall_overwrite(golden):
    """utils.jl:43-52: on wall death the head overwrites the wall with 1."""
    fx = golden["bson"]
    b = np.array(fx["board_final_rowmajor"])
    for r, c in fx["snake_1based"]:
        assert b[r - 1, c - 1] == 1
    assert any(b[r - 1, c - 1] == 1 and (r in (1, 10) or c in (1, 10)) for r, c in fx["snake_1based"])


def _replay(fx, n_frames):
    ob = oracle.OracleBatch(1, 10, n_frames)
    boards = fx["boards_cells"]
    first = n_frames  # index of b1 in the decoded history
    rewards, dones = [], []
    for t, a in enumerate(fx["act_idx"]):
        out = ob.step(np.array([a], np.uint8))
        assert out["status"] == 0
        assert np.array_equal(out["frames"][0, -1], boards[first + t]), f"step {t + 1}"
        # s_t / s'_t frames (utils.jl:141-149): b_{t-C} .. b_t with b_{-1} = b_0
        for f in range(n_frames + 1):
            k = first + t - n_frames + f
            assert np.array_equal(out["frames"][0, f], boards[max(k, n_frames - 1)])
        rewards.append(float(out["reward"][0]))
        dones.append(bool(out["done"][0]))
    return rewards, dones


def test_gif_double3_replays_every_frame(golden):
    fx = golden["double3"]
    assert fx["boards_cells"].shape == (240, 100) and len(fx["act_idx"]) == 237
    rewards, dones = _replay(fx, 2)
    assert sum(r == 1.0 for r in rewards) == 33          # README.md:54-58 score 33
    assert dones[-1] and not any(dones[:-1])             # ends in a wall collision
    ep = np.float32(0)
    for r in rewards:
        ep = np.float32(ep + np.float32(r))
    assert ep == np.float32(29.969957)                   # sequential Float32 sum (utils.jl:207)


def test_gif_vanilla_replays_every_frame(golden):
    fx = golden["vanilla1"]
    assert fx["boards_cells"].shape == (130, 100) and len(fx["act_idx"]) == 129
    rewards, dones = _replay(fx, 1)
    assert sum(r == 1.0 for r in rewards) == 8 and not any(dones)


def test_vanilla_qnet_greedy_kat(golden):
    """BSON vanilla weights + restated forward (kernel flip, column-major
    flatten) reproduce all 129 greedy actions of the vanilla GIF."""
    p = golden["vanilla_params"]
    assert p.size == oracle.qnet_nparams(10, 1) == golden["bson"]["qnet_nparams"] == 181251
    fx = golden["vanilla1"]
    states = fx["boards_cells"][:129].astype(np.float64)[:, None, :]
    q = oracle.qnet_forward(10, 1, p, states)
    assert (q.argmax(1) == fx["act_idx"]).all()
    np.testing.assert_allclose(q, golden["vanilla_q"], rtol=0, atol=1e-12)


def test_param_counts():
    assert oracle.qnet_nparams(10, 2) == 181395
    assert oracle.qnet_nparams(12, 2) == 279699
    assert oracle.qnet_nparams(20, 2) == 1000595


def test_backward_finite_difference():
    """The oracle backward (unpinned against the reference) agrees with
    central finite differences of its own forward."""
    rng = np.random.default_rng(0)
    bs, C = 8, 2
    P = oracle.qnet_nparams(bs, C)
    p = (rng.standard_normal(P) * 0.1).astype(np.float32)
    x = rng.integers(-1, 3, size=(3, C, bs * bs)).astype(np.float64)
    dq = rng.standard_normal((3, 3))
    g = oracle.qnet_backward(bs, C, p, x, dq)
    for i in rng.choice(P, 25, replace=False):
        h = 1e-3
        pp, pm = p.copy(), p.copy()
        pp[i] += h
        pm[i] -= h
        hp = float(np.float32(p[i] + h) - p[i])
        hm = float(p[i] - np.float32(p[i] - h))
        fd = ((oracle.qnet_forward(bs, C, pp, x) * dq).sum() - (oracle.qnet_forward(bs, C, pm, x) * dq).sum()) / (hp + hm)
        assert abs(fd - g[i]) <= 1e-4 * max(1.0, abs(g[i])), (i, fd, g[i])


def test_welford_matches_two_pass():
    rng = np.random.default_rng(1)
    D = rng.standard_normal((7, 50)) + 3.0
    Dc, mean, var = oracle.welford_center(D)
    np.testing.assert_allclose(mean, D.mean(0), rtol=1e-13)
    np.testing.assert_allclose(var, D.var(0, ddof=1), rtol=1e-12)
    np.testing.assert_allclose(Dc, D - mean, rtol=0, atol=1e-13)
    G = oracle.gram(Dc)
    np.testing.assert_allclose(G, Dc @ Dc.T, rtol=1e-12)
