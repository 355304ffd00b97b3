"""DQNModel on the GPU (structs.jl:120-147) and update_target_net!
(utils.jl:174-177).

Parameters cross the boundary in `Flux.destructure` order (per layer the
weight then the bias, each column-major), so a reference checkpoint's flat
vector loads unchanged (see tests/golden/vanilla_qnet_params.npy).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import DeviceArray, call, ptr, vp


def deep_nparams(board_size: int, n_frames: int) -> int:
    """Parameter count of the configs[2] net: 1,097,731 at bs=20, 2 frames."""
    wo = board_size - 5
    return ((9 * n_frames * 32 + 32) + (9 * 32 * 32 + 32) + (9 * 32 * 64 + 64) + (36 * 64 * 64 + 64)
            + (wo * wo * 64 * 64 + 64) + (64 * 3 + 3))


def nparams(board_size: int, n_frames: int) -> int:
    """Q-net parameter count: 279,699 at bs=12, 2 frames."""
    wo = board_size - 5
    return (9 * n_frames * 16 + 16) + (9 * 16 * 32 + 32) + (36 * 32 * 64 + 64) + (wo * wo * 64 * 64 + 64) + (64 * 3 + 3)


class DQNModel:
    """structs.jl:127 `DQNModel(board_size=10, n_actions=3; lr=0.0005)`.

    Weights: Flux glorot_uniform (zero biases) drawn from a counter RNG with
    `seed` (the reference uses Julia's unseeded global RNG); t_net starts as
    a copy of q_net; RMSProp(lr, rho=0.9, eps=1e-8)."""

    def __init__(self, board_size: int = 10, n_actions: int = 3, *, n_frames: int = 2, lr: float = 0.0005,
                 rho: float = 0.9, eps: float = 1e-8, seed: int = 1234, deep: bool = False):
        """deep=True: the deeper bf16 conv Q-net of BASELINE configs[2]
        (include/snakehip.h snk_dqn_create_deep; board side 10, 12 or 20)."""
        if n_actions != 3:
            raise ValueError("the reference Q-net has 3 outputs (structs.jl:134)")
        self.board_size, self.n_frames, self.n_actions = int(board_size), int(n_frames), 3
        self.lr, self.rho, self.eps = float(lr), float(rho), float(eps)
        self.deep = bool(deep)
        h = vp()
        call("snk_dqn_create_deep" if self.deep else "snk_dqn_create", C.byref(h), self.board_size, self.n_frames,
             self.lr, self.rho, self.eps, int(seed))
        self._h = h
        n = C.c_int64(0)
        call("snk_dqn_nparams", h, C.byref(n))
        self.P = n.value

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.snk_dqn_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    # Flux.destructure / restructure
    def get_params(self, which: int = _lib.SNK_NET_Q) -> np.ndarray:
        out = np.zeros(self.P, np.float32)
        call("snk_dqn_get_params", self._h, which, ptr(out))
        return out

    def set_params(self, flat, which: int = _lib.SNK_NET_Q) -> None:
        flat = np.ascontiguousarray(flat, np.float32)
        assert flat.size == self.P, (flat.size, self.P)
        call("snk_dqn_set_params", self._h, which, ptr(flat))

    def buffer_ptr(self, which: int) -> int:
        p = vp()
        call("snk_dqn_buffer_ptr", self._h, which, C.byref(p))
        return p.value

    def flux_index(self) -> np.ndarray:
        """perm[j] = the Flux.destructure index of packed position j (the
        device layout behind buffer_ptr and the trainer's gradient trace):
        flux[perm] = packed. Found by round-tripping 0..P-1 through the
        gradient slot, which is restored afterwards."""
        keep = self.grad
        self.set_params(np.arange(self.P, dtype=np.float32), _lib.SNK_NET_GRAD)   # exact below 2^24
        perm = _lib.view_numpy(self.buffer_ptr(_lib.SNK_NET_GRAD), self.P, np.float32).astype(np.int64)
        self.set_params(keep, _lib.SNK_NET_GRAD)
        return perm

    def forward(self, x, which: int = _lib.SNK_NET_Q) -> np.ndarray:
        """Chain forward on Float32 states [B, C, bs*bs] (Julia (bs,bs,C,B)
        memory) -> Q [B, 3]."""
        x = np.ascontiguousarray(x, np.float32)
        B = x.shape[0]
        dx = DeviceArray.from_host(x.reshape(B, -1))
        dq = DeviceArray((B, 3), np.float32)
        call("snk_dqn_forward", self._h, which, dx.ptr, B, dq.ptr)
        return dq.numpy()

    __call__ = forward

    def q_env(self, game, which: int = _lib.SNK_NET_Q) -> np.ndarray:
        dq = DeviceArray((game.n_envs, 3), np.float32)
        call("snk_dqn_forward_env", self._h, which, game.handle, dq.ptr)
        return dq.numpy()

    def loss_grad(self, rpb, idx, B: int, gamma: float = 0.97) -> float:
        loss = C.c_double(0)
        call("snk_dqn_loss_grad", self._h, rpb.handle, idx.ptr, B, gamma, C.byref(loss))
        return loss.value

    def loss_grad_batch(self, batch: dict, gamma: float = 0.97) -> float:
        """utils.jl:448-464 on explicit stack_exp tensors (host arrays)."""
        B = batch["states"].shape[0]
        arrs = [DeviceArray.from_host(np.ascontiguousarray(batch[k], t)) for k, t in
                (("states", np.float32), ("actions", np.int32), ("rewards", np.float32),
                 ("next_states", np.float32), ("dones", np.uint8), ("suicidal_mask", np.uint8))]
        loss = C.c_double(0)
        call("snk_dqn_loss_grad_batch", self._h, *[a.ptr for a in arrs], B, gamma, C.byref(loss))
        return loss.value

    def apply_grad(self) -> None:
        call("snk_dqn_apply_grad", self._h)

    def update(self, rpb, idx, B: int, gamma: float = 0.97) -> float:
        loss = C.c_double(0)
        call("snk_dqn_update", self._h, rpb.handle, idx.ptr, B, gamma, C.byref(loss))
        return loss.value

    def train_relu_decisions(self, B: int) -> np.ndarray:
        """The relu decisions (output > 0) of q_net in the last training forward
        over B samples, [B, n] uint8 in the oracle's order: a1 | a2 | a3
        channel-major (position = i + j*side) | h1. Test infrastructure (kink-aware
        gradient parity, oracle.dqn_loss_grad_kinks)."""
        bs, wo = self.board_size, self.board_size - 5
        parts = []
        for layer, (npos, ch) in enumerate(((bs * bs, 16), (bs * bs, 32), (wo * wo, 64), (1, 64))):
            a = np.empty((B, npos, ch), np.float32)
            call("snk_dqn_train_activations", self._h, layer, ptr(a), a.size)
            parts.append((a > 0).transpose(0, 2, 1).reshape(B, -1))
        return np.ascontiguousarray(np.concatenate(parts, axis=1), np.uint8)

    @property
    def grad(self) -> np.ndarray:
        return self.get_params(_lib.SNK_NET_GRAD)


def update_target_net_(model: DQNModel) -> None:
    """utils.jl:174-177: t_net <- copy of q_net."""
    call("snk_dqn_sync_target", model.handle)
