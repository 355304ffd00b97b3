"""BSON checkpoint interop (utils.jl:408-418 save_trainer / load_trainer).

CPU: the reference's own checkpoint trainers/very_long_training1.bson (read
as data here, where /root/reference exists; skipped elsewhere) parses to the
values the committed fixtures hold (tests/golden/make_fixtures.py decoded
them independently): the q_net weights bit-exact in Flux.destructure order,
t_net == q_net, the schedule fields and the history lengths.
GPU: load_trainer on a BSON.jl-shaped checkpoint written from a device
model restores q_net / t_net bit-exact and the schedule fields.
"""
import os

import numpy as np
import pytest

REF_BSON = "/root/reference/trainers/very_long_training1.bson"


@pytest.mark.skipif(not os.path.exists(REF_BSON), reason="reference checkpoint not present (GPU box)")
def test_read_reference_checkpoint(golden):
    from snake_amd.bsonio import read_trainer
    d = read_trainer(REF_BSON)
    fx = golden["bson"]
    assert d["board_size"] == fx["board_size"] == 10
    assert d["n_frames"] == 1 and d["n_actions"] == 3
    assert d["layer_shapes"] == fx["qnet_layer_shapes"]
    assert np.array_equal(d["q_params"], golden["vanilla_params"])
    assert np.array_equal(d["t_params"], d["q_params"]) == fx["tnet_equals_qnet"]
    assert list(d["rmsprop"]) == fx["rmsprop_eta_rho_eps"]
    for k in ("n_batches", "target_update_rate", "epsilon", "epsilon_end", "decay"):
        assert d[k] == fx[k], k
    assert d["losses"].size == fx["n_losses"] and d["episode_rewards"].size == fx["n_episode_rewards"]
    assert abs(float(d["losses"][-5000:].astype(np.float64).mean()) - fx["mean_last5000_loss"]) < 1e-12
    assert float(d["episode_rewards"].max()) == np.float32(fx["max_episode_reward"])


# ---- a BSON.jl-shaped writer for the GPU round trip (same tags as BSON.jl emits)
def _dtype(name):
    return {"tag": "datatype", "name": ["Core", name], "params": []}


def _arr(a, name):
    a = np.asarray(a)
    return {"tag": "array", "type": _dtype(name), "size": list(a.shape),
            "data": np.asfortranarray(a).tobytes(order="F")}


def _bits(v, dt, name):
    return {"tag": "struct", "type": _dtype(name), "data": np.array([v], dt).tobytes()}


def _struct(mod, name, fields):
    return {"tag": "struct", "type": {"tag": "datatype", "name": [mod, name], "params": []}, "data": fields}


def _chain_doc(flat, bs, C):
    wo = bs - 5
    shapes = [(3, 3, C, 16), (16,), (3, 3, 16, 32), (32,), (6, 6, 32, 64), (64,), (64, wo * wo * 64), (64,),
              (3, 64), (3,)]
    arrs, o = [], 0
    for sh in shapes:
        n = int(np.prod(sh))
        arrs.append(flat[o:o + n].reshape(sh, order="F"))
        o += n
    assert o == flat.size
    conv = [_struct("Flux", "Conv", ["relu", _arr(arrs[2 * i], "Float32"), _arr(arrs[2 * i + 1], "Float32")])
            for i in range(3)]
    dense = [_struct("Flux", "Dense", [_arr(arrs[6 + 2 * i], "Float32"), _arr(arrs[7 + 2 * i], "Float32"), "relu"])
             for i in range(2)]
    layers = {"tag": "tuple", "data": conv[:3] + ["flatten"] + dense}
    return _struct("Flux", "Chain", [layers])


@pytest.mark.gpu
def test_load_trainer_roundtrip(snk, tmp_path):
    import bson
    bs, C = 12, 2
    src = snk.DQNModel(bs, 3, n_frames=C, seed=77)
    q = src.get_params()
    t = (q * np.float32(0.5)).astype(np.float32)
    board = np.zeros((bs, bs), np.int64)
    game = _struct("Main", "SnakeGame", [bs, C, _arr(board, "Int64")])
    model = _struct("Main", "DQNModel", [_chain_doc(q, bs, C), _chain_doc(t, bs, C),
                                         _struct("Flux.Optimise", "RMSProp", [0.0005, 0.9, 1e-08, {}])])
    tr = _struct("Main", "Trainer", [game, model, None, 1234, 500, _bits(0.25, np.float32, "Float32"),
                                     _bits(0.05, np.float32, "Float32"), _bits(1e-6, np.float32, "Float32"), True,
                                     _arr(np.array([0.5, 0.25], np.float32), "Float32"),
                                     _arr(np.array([1.0, -1.0, 3.0], np.float32), "Float32")])
    path = str(tmp_path / "ckpt.bson")
    with open(path, "wb") as f:
        f.write(bson.encode({"tr": tr, "_backrefs": []}))
    tl = snk.load_trainer(path, capacity=1000)
    assert tl.model.board_size == bs and tl.model.n_frames == C
    assert np.array_equal(tl.model.get_params(), q)
    assert np.array_equal(tl.model.get_params(snk.SNK_NET_TARGET), t)
    assert tl.n_batches == 1234 and tl.target_update_rate == 500
    assert np.float32(tl.epsilon) == np.float32(0.25) and np.float32(tl.decay) == np.float32(1e-6)
    assert tl.episode_losses == [0.5, 0.25] and tl.episode_rewards == [1.0, -1.0, 3.0]
