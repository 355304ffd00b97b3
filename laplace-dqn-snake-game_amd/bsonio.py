"""load_trainer (utils.jl:414-418): Julia BSON.jl checkpoints of the reference's
Trainer (structs.jl:151-175), read as data for warm starts.

A BSON.jl file is ordinary BSON (decoded with pymongo's `bson`, nothing in
the file is executed); Julia objects are tagged documents: {"tag": "struct",
"type": ..., "data": [fields in declaration order]}, {"tag": "array", "type",
"size", "data": raw little-endian bytes, column-major}, and {"tag":
"backref", "ref": k} into the top-level "_backrefs" list.

What is taken from the file:
  * q_net / t_net: the Flux Chain's Conv / Dense weights and biases,
    flattened in Flux.destructure order (per layer weight then bias, each
    column-major), which is the order DQNModel.set_params takes;
  * board side: from the game's board matrix (its shape, not a field index:
    the SnakeGame struct gained fields between the reference's versions);
  * frames: conv1's input channels; RMSProp eta/rho/eps: model.opt;
  * n_batches, target_update_rate, epsilon, epsilon_end, decay, losses,
    episode_rewards: Trainer fields 3..10 (structs.jl:153-163).
The replay buffer is not restored (the reference saves it separately,
utils.jl:488).
"""
from __future__ import annotations

import os

import numpy as np

_DTYPES = {"Core.Float32": np.float32, "Core.Float64": np.float64, "Core.Int64": np.int64,
           "Core.Bool": np.bool_, "Core.UInt8": np.uint8}


class JuliaBSON:
    """A decoded BSON.jl document with backref resolution."""

    def __init__(self, path: str):
        try:
            import bson  # pymongo's decoder
        except ImportError as e:  # pragma: no cover - environment without pymongo
            raise ImportError("reading Julia BSON checkpoints needs pymongo's `bson` module") from e
        with open(path, "rb") as f:
            self.doc = bson.decode(f.read())
        self.backrefs = self.doc.get("_backrefs", [])

    def res(self, x):
        while isinstance(x, dict) and x.get("tag") == "backref":
            x = self.backrefs[x["ref"] - 1]
        return x

    def type_name(self, x) -> str:
        return ".".join(self.res(self.res(x)["type"])["name"])

    def array(self, x) -> np.ndarray:
        x = self.res(x)
        if x.get("tag") != "array":
            raise ValueError(f"not a Julia array: tag {x.get('tag')!r}")
        name = ".".join(self.res(x["type"])["name"])
        if name not in _DTYPES:
            raise ValueError(f"unsupported Julia element type {name}")
        size = x["size"]
        return np.frombuffer(x["data"], dtype=_DTYPES[name]).reshape(size, order="F")

    def scalar(self, x, dtype):
        x = self.res(x)
        if isinstance(x, dict):   # bits types are stored as {"tag": "struct", "data": raw bytes}
            return np.frombuffer(x["data"], dtype)[0].item()
        return x


def _chain(jb: JuliaBSON, chain) -> tuple[np.ndarray, list]:
    """Flux.destructure of a Chain of Conv / Dense layers (Flux.flatten skipped)."""
    layers = jb.res(jb.res(chain)["data"][0])["data"]
    parts = []
    for layer in layers:
        layer = jb.res(layer)
        if not isinstance(layer, dict) or "type" not in layer:   # Flux.flatten (a function)
            continue
        t = jb.type_name(layer)
        if t == "Flux.Conv":      # fields: σ, weight, bias, stride, pad, dilation, groups
            parts += [jb.array(layer["data"][1]), jb.array(layer["data"][2])]
        elif t == "Flux.Dense":   # fields: weight, bias, σ
            parts += [jb.array(layer["data"][0]), jb.array(layer["data"][1])]
    flat = np.concatenate([np.asarray(a, np.float32).ravel(order="F") for a in parts])
    return flat, [list(a.shape) for a in parts]


def read_trainer(path: str) -> dict:
    """The Trainer of a `@save path tr` checkpoint (utils.jl:408-412) as plain data."""
    jb = JuliaBSON(path)
    tr = jb.res(jb.doc["tr"])
    f = tr["data"]
    game, model = jb.res(f[0]), jb.res(f[1])
    board = None
    for x in game["data"]:
        x = jb.res(x)
        if isinstance(x, dict) and x.get("tag") == "array" and len(x["size"]) == 2 and x["size"][0] == x["size"][1]:
            board = jb.array(x)
            break
    if board is None:
        raise ValueError("no square board matrix in the checkpoint's game")
    q, shapes = _chain(jb, model["data"][0])
    t, _ = _chain(jb, model["data"][1])
    opt = jb.res(model["data"][2])
    eta, rho, eps = (float(v) for v in opt["data"][:3])
    return {
        "board_size": int(board.shape[0]),
        "n_frames": int(shapes[0][2]),          # conv1 weight (3, 3, C, 16)
        "n_actions": int(shapes[-1][0]),        # Dense(64, n_actions) weight (n_actions, 64)
        "layer_shapes": shapes,
        "q_params": q,
        "t_params": t,
        "rmsprop": (eta, rho, eps),
        "n_batches": int(jb.scalar(f[3], np.int64)),
        "target_update_rate": int(jb.scalar(f[4], np.int64)),
        "epsilon": float(jb.scalar(f[5], np.float32)),
        "epsilon_end": float(jb.scalar(f[6], np.float32)),
        "decay": float(jb.scalar(f[7], np.float32)),
        "save": bool(jb.scalar(f[8], np.bool_)),
        "losses": np.asarray(jb.array(f[9]), np.float32),
        "episode_rewards": np.asarray(jb.array(f[10]), np.float32),
    }


def load_trainer(name: str, *, directory: str = "./trainers/", n_envs: int = 1, capacity: int = 50000,
                 batch_size: int = 64, seed: int = 1234):
    """utils.jl:414-418 `load_trainer(name)` ("./trainers/" * name * ".bson",
    or a path ending in .bson): a Trainer whose q_net / t_net hold the
    checkpoint's weights and whose schedule fields continue from it
    (epsilon, decay, ...); tr.losses / tr.episode_rewards histories come back
    as tr.episode_losses / tr.episode_rewards."""
    from .qnet import DQNModel
    from .trainer import Trainer
    from ._lib import SNK_NET_TARGET

    path = name if name.endswith(".bson") else os.path.join(directory, name + ".bson")
    d = read_trainer(path)
    if d["n_actions"] != 3:
        raise ValueError(f"checkpoint Q-net has {d['n_actions']} outputs; the reference net has 3")
    eta, rho, eps = d["rmsprop"]
    model = DQNModel(d["board_size"], 3, n_frames=d["n_frames"], lr=eta, rho=rho, eps=eps, seed=seed)
    if model.P != d["q_params"].size:
        raise ValueError(f"checkpoint has {d['q_params'].size} parameters, the model {model.P}")
    model.set_params(d["q_params"])
    model.set_params(d["t_params"], SNK_NET_TARGET)
    tr = Trainer(n_batches=d["n_batches"], target_update_rate=d["target_update_rate"], epsilon=d["epsilon"],
                 epsilon_end=d["epsilon_end"], decay=d["decay"], save=d["save"], model=model, n_envs=n_envs,
                 board_size=d["board_size"], n_frames=d["n_frames"], capacity=capacity, batch_size=batch_size,
                 seed=seed)
    tr.episode_losses = [float(v) for v in d["losses"]]
    tr.episode_rewards = [float(v) for v in d["episode_rewards"]]
    return tr
