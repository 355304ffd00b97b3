#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the
reference's own DATA files (run in the build container, where
/root/reference exists; the GPU box never runs this).

Inputs (read-only, parsed as data — nothing is executed from them):
  /root/reference/trainers/very_long_training1.bson   (BSON via pymongo's
      `bson` decoder; Julia BSON.jl tagging resolved by hand)
  /root/reference/trainer_gifs/very_long_double_training3.gif
  /root/reference/trainer_gifs/very_long_training1.gif     (Pillow)

Outputs:
  bson_vanilla.json          food_list, Xoshiro state words, final board/snake,
                             RMSProp fields, training-curve statistics
  vanilla_qnet_params.npy    q_net flat params in Flux.destructure order (f32)
  gif_double3.npz            240 decoded boards (2-frame best game) + actions
  gif_vanilla1.npz           130 decoded boards (1-frame vanilla game) + actions
  vanilla_q_fp64.npy         oracle fp64 Q-values of the 129 vanilla states
                             (regression vector; the pin is the argmax KAT)

Actions are recovered from the boards: at each step exactly one of the three
available actions (utils.jl:7-10) reproduces the next decoded frame under the
oracle's step! restatement; the script asserts that uniqueness.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402


# ------------------------------------------------------------------ BSON
def load_bson(path):
    import bson
    with open(path, "rb") as f:
        d = bson.decode(f.read())
    br = d["_backrefs"]

    def res(x):
        while isinstance(x, dict) and x.get("tag") == "backref":
            x = br[x["ref"] - 1]
        return x

    return d, res


def jarray(x, res):
    x = res(x)
    assert x["tag"] == "array", x.get("tag")
    t = res(x["type"])
    name = ".".join(t["name"])
    dt = {"Core.Float32": np.float32, "Core.Int64": np.int64, "Core.Float64": np.float64,
          "Main.Base.IteratorsMD.CartesianIndex": np.int64}[name]
    a = np.frombuffer(x["data"], dtype=dt)
    size = x["size"]
    if name.endswith("CartesianIndex"):
        return a.reshape(-1, 2)                      # (row, col) per entry
    return a.reshape(size, order="F")


def u64(x, res):
    x = res(x)
    return int.from_bytes(x["data"], "little")


def f32(x, res):
    x = res(x)
    return float(np.frombuffer(x["data"], np.float32)[0])


def bson_fixture():
    d, res = load_bson(os.path.join(REF, "trainers", "very_long_training1.bson"))
    tr = res(d["tr"])
    game, model = res(tr["data"][0]), res(tr["data"][1])
    gd = game["data"]
    board = jarray(gd[0], res)
    snake = jarray(gd[1], res)
    food = jarray(gd[13], res)
    rng = res(gd[9])
    rng_words = [u64(w, res) for w in rng["data"]]

    def chain_params(chain):
        layers = res(res(chain)["data"][0])["data"]
        out = []
        for layer in layers:
            layer = res(layer)
            tname = ".".join(res(layer["type"])["name"])
            if tname == "Flux.Conv":
                out += [jarray(layer["data"][1], res), jarray(layer["data"][2], res)]
            elif tname == "Flux.Dense":
                out += [jarray(layer["data"][0], res), jarray(layer["data"][1], res)]
        shapes = [list(a.shape) for a in out]
        flat = np.concatenate([a.ravel(order="F") for a in out]).astype(np.float32)
        return flat, shapes

    qp, shapes = chain_params(model["data"][0])
    tp, _ = chain_params(model["data"][1])
    opt = res(model["data"][2])
    losses = jarray(tr["data"][9], res).astype(np.float64)
    ep_rewards = jarray(tr["data"][10], res).astype(np.float64)
    fx = {
        "source": "reference trainers/very_long_training1.bson (data fields only)",
        "board_size": int(gd[10]),
        "food_list_1based": food.tolist(),
        "food_rng_state_s0_s4_hex": ["%016x" % w for w in rng_words],
        "board_final_rowmajor": board.tolist(),
        "snake_1based": snake.tolist(),
        "score": int(gd[4]),
        "lost": bool(gd[11]),
        "qnet_layer_shapes": shapes,
        "qnet_nparams": int(qp.size),
        "tnet_equals_qnet": bool(np.array_equal(qp, tp)),
        "rmsprop_eta_rho_eps": [float(v) for v in opt["data"][:3]],
        "n_batches": int(tr["data"][3]),
        "target_update_rate": int(tr["data"][4]),
        "epsilon": f32(tr["data"][5], res),
        "epsilon_end": f32(tr["data"][6], res),
        "decay": f32(tr["data"][7], res),
        "n_losses": int(losses.size),
        "n_episode_rewards": int(ep_rewards.size),
        "mean_last5000_loss": float(losses[-5000:].mean()),
        "mean_last5000_episode_reward": float(ep_rewards[-5000:].mean()),
        "max_episode_reward": float(ep_rewards.max()),
    }
    return fx, qp


# ------------------------------------------------------------------ GIFs
COLORS = {(0, 0, 0): -1, (255, 255, 255): 0}


def decode_gif(path, bs=10, cell=36, y0=12, x0=131):
    from PIL import Image
    im = Image.open(path)
    boards = []
    for k in range(im.n_frames):
        im.seek(k)
        a = np.asarray(im.convert("RGB")).astype(int)
        b = np.zeros((bs, bs), np.int8)
        for i in range(bs):
            for j in range(bs):
                r, g, bb = a[y0 + i * cell + cell // 2, x0 + j * cell + cell // 2]
                if (r, g, bb) in COLORS:
                    v = COLORS[(r, g, bb)]
                elif g > 200 and r < 60 and bb < 60:
                    v = 1
                elif r > 200 and g < 60 and bb < 60:
                    v = 2
                else:
                    raise ValueError(f"frame {k} cell {(i, j)} colour {(r, g, bb)}")
                b[i, j] = v
        boards.append(b)
    return np.stack(boards)


def to_cells(b_rowmajor):
    """[.., bs, bs] row-major board[i][j] -> [.., bs*bs] column-major cells."""
    b = np.asarray(b_rowmajor)
    return np.swapaxes(b, -1, -2).reshape(*b.shape[:-2], -1)


def recover_actions(boards_cells, n_frames, bs=10):
    """Search the unique available-action index per step that reproduces the
    next decoded board under the oracle's step!. Returns (act_idx, dirs)."""
    first = n_frames - 1                 # history = [b0]*n_frames + [b1..]
    targets = boards_cells[first + 1:]
    if n_frames == 2:
        targets = targets[:-1]           # trailing copy of the final board (utils.jl:223)
    acts, dirs = [], []
    for t in range(len(targets)):
        ok = []
        for a in range(3):
            ob = oracle.OracleBatch(1, bs, n_frames)
            for p in acts:
                ob.step(np.array([p], np.uint8), want_frames=False)
            out = ob.step(np.array([a], np.uint8), want_frames=True)
            nb = out["frames"][0, -1]
            if np.array_equal(nb, targets[t]):
                ok.append((a, int(out["dir"][0]), bool(out["done"][0])))
        if len(ok) != 1:
            raise RuntimeError(f"step {t + 1}: {len(ok)} actions reproduce the frame")
        acts.append(ok[0][0])
        dirs.append(ok[0][1])
        if ok[0][2]:
            assert t == len(targets) - 1, "game lost before the last decoded frame"
    return np.array(acts, np.uint8), np.array(dirs, np.uint8)


def main():
    fx, qp = bson_fixture()
    with open(os.path.join(HERE, "bson_vanilla.json"), "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    np.save(os.path.join(HERE, "vanilla_qnet_params.npy"), qp)
    print("bson: P =", qp.size, "food[:4] =", fx["food_list_1based"][:4])

    letters = "UDLR"
    for name, nf in (("very_long_double_training3", 2), ("very_long_training1", 1)):
        rows = decode_gif(os.path.join(REF, "trainer_gifs", name + ".gif"))
        cells = to_cells(rows)
        acts, dirs = recover_actions(cells, nf)
        out = "gif_double3.npz" if nf == 2 else "gif_vanilla1.npz"
        np.savez_compressed(os.path.join(HERE, out), boards_cells=cells, act_idx=acts, dirs=dirs,
                            n_frames=np.int32(nf), board_size=np.int32(10))
        print(name, "frames", len(rows), "steps", len(acts), "".join(letters[d] for d in dirs)[:40], "...")

    # fp64 oracle Q for the 129 vanilla states (1 frame, bs=10): state_t = b_t
    v = np.load(os.path.join(HERE, "gif_vanilla1.npz"))
    states = v["boards_cells"][:len(v["act_idx"])].astype(np.float64)[:, None, :]
    q = oracle.qnet_forward(10, 1, qp, states)
    np.save(os.path.join(HERE, "vanilla_q_fp64.npy"), q)
    print("vanilla greedy KAT:", int((q.argmax(1) == v["act_idx"]).sum()), "/", len(q))


if __name__ == "__main__":
    main()
