"""ctypes wrapper around the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker. The product package
(laplace-dqn-snake-game_amd/) never imports this module.

See snake_oracle.h for what each function restates (reference file:line) and
how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

F32P = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
F64P = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
I32P = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
U8P = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
I8P = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = [os.path.join(_HERE, f) for f in ("snake_oracle.c", "snake_oracle.h")]
    if not os.path.exists(path) or any(os.path.getmtime(s) > os.path.getmtime(path) for s in src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return path


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    L = C.CDLL(build())
    L.orc_julia_xoshiro_seed.argtypes = [C.c_uint32, U64P]
    L.orc_food_list.argtypes = [C.c_int, C.c_uint32, C.c_int, I32P, U64P]
    L.orc_game_sizeof.restype = C.c_int
    L.orc_batch_create.restype = C.c_void_p
    L.orc_batch_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, I32P, C.c_int]
    L.orc_batch_destroy.argtypes = [C.c_void_p]
    L.orc_batch_step.restype = C.c_int
    L.orc_batch_step.argtypes = [C.c_void_p, U8P, F32P, U8P, U8P, U8P, U8P, C.c_void_p]
    L.orc_batch_boards.argtypes = [C.c_void_p, I8P]
    L.orc_batch_scalars.argtypes = [C.c_void_p, I32P, I32P, I32P, I32P, F32P]
    L.orc_batch_states.argtypes = [C.c_void_p, I8P]
    L.orc_splitmix64.restype = C.c_uint64
    L.orc_splitmix64.argtypes = [C.c_uint64]
    L.orc_synth_action.restype = C.c_uint32
    L.orc_synth_action.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    L.orc_qnet_nparams.restype = C.c_int64
    L.orc_qnet_nparams.argtypes = [C.c_int, C.c_int]
    L.orc_qnet_forward.argtypes = [C.c_int, C.c_int, F32P, C.c_int, F64P, F64P]
    L.orc_qnet_backward.argtypes = [C.c_int, C.c_int, F32P, C.c_int, F64P, F64P, F64P]
    L.orc_dqn_loss_grad.restype = C.c_double
    L.orc_dqn_loss_grad.argtypes = [C.c_int, C.c_int, F32P, F32P, C.c_int, F64P, I32P, F32P, F64P,
                                    U8P, U8P, C.c_double, F64P, F64P]
    L.orc_qnet_relu_count.restype = C.c_int64
    L.orc_qnet_relu_count.argtypes = [C.c_int, C.c_int]
    L.orc_dqn_loss_grad_ex.restype = C.c_double
    L.orc_dqn_loss_grad_ex.argtypes = [C.c_int, C.c_int, F32P, F32P, C.c_int, F64P, I32P, F32P, F64P,
                                       U8P, U8P, C.c_double, F64P, F64P, C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_deep_nparams.restype = C.c_int64
    L.orc_deep_nparams.argtypes = [C.c_int, C.c_int]
    L.orc_deep_forward.argtypes = [C.c_int, C.c_int, F32P, C.c_int, F64P, F64P]
    L.orc_deep_backward.argtypes = [C.c_int, C.c_int, F32P, C.c_int, F64P, F64P, F64P]
    L.orc_deep_loss_grad.restype = C.c_double
    L.orc_deep_loss_grad.argtypes = [C.c_int, C.c_int, F32P, F32P, C.c_int, F64P, I32P, F32P, F64P,
                                     U8P, U8P, C.c_double, F64P, F64P]
    L.orc_rmsprop.argtypes = [C.c_int64, F32P, F32P, F32P, C.c_float, C.c_float, C.c_float]
    L.orc_welford_center.argtypes = [C.c_int64, C.c_int, F64P, F64P, F64P]
    L.orc_gram.argtypes = [C.c_int64, C.c_int, F64P, F64P]
    _LIB = L
    return L


_FAST = None


def fast():
    """libcpufast.so (cpu_fast.cpp): the optimised multi-threaded CPU
    restatement bench.py times as cpu_baseline. Same test-only status."""
    global _FAST
    if _FAST is not None:
        return _FAST
    path = os.path.join(_HERE, "libcpufast.so")
    if not os.path.exists(path) or os.path.getmtime(os.path.join(_HERE, "cpu_fast.cpp")) > os.path.getmtime(path):
        subprocess.run(["make", "-C", _HERE, "-s", "libcpufast.so"], check=True)
    L = C.CDLL(path)
    L.cpuf_env_create.restype = C.c_void_p
    L.cpuf_env_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, I32P, C.c_int]
    L.cpuf_env_destroy.argtypes = [C.c_void_p]
    L.cpuf_env_step.argtypes = [C.c_void_p, U8P, F32P, U8P, U8P, C.c_int]
    L.cpuf_env_boards.argtypes = [C.c_void_p, I8P]
    L.cpuf_qnet_forward.argtypes = [C.c_int, C.c_int, F32P, C.c_int, F32P, F32P, C.c_int]
    L.cpuf_loss_grad.restype = C.c_double
    L.cpuf_loss_grad.argtypes = [C.c_int, C.c_int, F32P, F32P, C.c_int, F32P, I32P, F32P, F32P, U8P, U8P, F32P,
                                 C.c_int]
    L.cpuf_bench.restype = C.c_double
    L.cpuf_bench.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, I32P, C.c_int,
                             F64P]
    L.cpuf_gram.restype = C.c_double
    L.cpuf_gram.argtypes = [C.c_int, C.c_int, F32P, F32P, C.c_int]
    L.cpuf_max_threads.restype = C.c_int
    _FAST = L
    return L


# ---------------------------------------------------------------- RNG / food
def xoshiro_seed(seed: int = 42) -> np.ndarray:
    st = np.zeros(5, np.uint64)
    lib().orc_julia_xoshiro_seed(seed, st)
    return st


def food_list(bs: int, seed: int = 42, n: int = 50):
    """structs.jl:70 — returns (cells int32[n] column-major 0-based, rng state after)."""
    cells = np.zeros(n, np.int32)
    st = np.zeros(4, np.uint64)
    lib().orc_food_list(bs, seed, n, cells, st)
    return cells, st


def synth_action(seed: int, env: int, step: int) -> int:
    return int(lib().orc_synth_action(seed, env, step))


def synth_actions(seed: int, n_envs: int, step: int) -> np.ndarray:
    L = lib()
    return np.array([L.orc_synth_action(seed, e, step) for e in range(n_envs)], np.uint8)


# ---------------------------------------------------------------- env
class OracleBatch:
    """N independent SnakeGame()s stepped in lockstep with auto-reset."""

    def __init__(self, n: int, bs: int = 10, n_frames: int = 2, max_hist: int = 500,
                 food: np.ndarray | None = None):
        if food is None:
            food, _ = food_list(bs)
        self.n, self.bs, self.C = n, bs, n_frames
        self.food = np.ascontiguousarray(food, np.int32)
        self._h = lib().orc_batch_create(n, bs, n_frames, max_hist, self.food, len(self.food))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_batch_destroy(self._h)
            self._h = None

    def step(self, act_idx: np.ndarray, want_frames: bool = True):
        n, nc = self.n, self.bs * self.bs
        act = np.ascontiguousarray(act_idx, np.uint8)
        out = dict(reward=np.zeros(n, np.float32), done=np.zeros(n, np.uint8),
                   mask=np.zeros((n, 3), np.uint8), dir=np.zeros(n, np.uint8),
                   prev_dir=np.zeros(n, np.uint8))
        frames = np.zeros((n, self.C + 1, nc), np.int8) if want_frames else None
        st = lib().orc_batch_step(self._h, act, out["reward"], out["done"], out["mask"], out["dir"],
                                  out["prev_dir"], frames.ctypes.data if want_frames else None)
        out["status"] = st
        out["frames"] = frames
        return out

    def boards(self) -> np.ndarray:
        b = np.zeros((self.n, self.bs * self.bs), np.int8)
        lib().orc_batch_boards(self._h, b)
        return b

    def states(self) -> np.ndarray:
        s = np.zeros((self.n, self.C, self.bs * self.bs), np.int8)
        lib().orc_batch_states(self._h, s)
        return s

    def scalars(self):
        n = self.n
        sc, ln, stp, pd = (np.zeros(n, np.int32) for _ in range(4))
        ep = np.zeros(n, np.float32)
        lib().orc_batch_scalars(self._h, sc, ln, stp, pd, ep)
        return dict(score=sc, len=ln, steps=stp, prev_dir=pd, episode_reward=ep)


# ---------------------------------------------------------------- Q-net
def qnet_nparams(bs: int, C: int) -> int:
    return int(lib().orc_qnet_nparams(bs, C))


def qnet_forward(bs: int, C: int, params: np.ndarray, x: np.ndarray) -> np.ndarray:
    """x: [B, C, bs*bs] (Julia (bs,bs,C,B) memory), returns fp64 Q [B, 3]."""
    x = np.ascontiguousarray(x, np.float64).reshape(-1, C * bs * bs)
    B = x.shape[0]
    q = np.zeros((B, 3), np.float64)
    lib().orc_qnet_forward(bs, C, np.ascontiguousarray(params, np.float32), B, x, q)
    return q


def qnet_backward(bs: int, C: int, params: np.ndarray, x: np.ndarray, dq: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float64).reshape(-1, C * bs * bs)
    B = x.shape[0]
    g = np.zeros(len(params), np.float64)
    lib().orc_qnet_backward(bs, C, np.ascontiguousarray(params, np.float32), B, x,
                            np.ascontiguousarray(dq, np.float64).reshape(B, 3), g)
    return g


def dqn_loss_grad(bs, C, q_params, t_params, s, a_idx, r, s_next, done, mask3, gamma=0.97):
    s = np.ascontiguousarray(s, np.float64).reshape(-1, C * bs * bs)
    B = s.shape[0]
    g = np.zeros(len(q_params), np.float64)
    tgt = np.zeros(B, np.float64)
    loss = lib().orc_dqn_loss_grad(bs, C, np.ascontiguousarray(q_params, np.float32),
                                   np.ascontiguousarray(t_params, np.float32), B, s,
                                   np.ascontiguousarray(a_idx, np.int32),
                                   np.ascontiguousarray(r, np.float32),
                                   np.ascontiguousarray(s_next, np.float64).reshape(B, -1),
                                   np.ascontiguousarray(done, np.uint8),
                                   np.ascontiguousarray(mask3, np.uint8).reshape(B, 3), gamma, g, tgt)
    return loss, g, tgt


def dqn_loss_grad_kinks(bs, C, q_params, t_params, s, a_idx, r, s_next, done, mask3, gamma=0.97, relu_in=None):
    """dqn_loss_grad with the q_net's relu decisions exposed: returns (loss,
    grad, relu decisions [B, n], margins [B, n]) where n = a1 | a2 | a3 | h1
    (channel-major per layer, orc_qnet_relu_count) and margin = z / sum|terms|.
    relu_in ([B, n] uint8) replaces the z > 0 decisions (the device's own, to
    check that a gradient difference is a kink decision and nothing else)."""
    s = np.ascontiguousarray(s, np.float64).reshape(-1, C * bs * bs)
    B = s.shape[0]
    n = int(lib().orc_qnet_relu_count(bs, C))
    g = np.zeros(len(q_params), np.float64)
    tgt = np.zeros(B, np.float64)
    dec = np.zeros((B, n), np.uint8)
    mg = np.zeros((B, n), np.float64)
    rin = None if relu_in is None else np.ascontiguousarray(relu_in, np.uint8).reshape(B, n)
    loss = lib().orc_dqn_loss_grad_ex(bs, C, np.ascontiguousarray(q_params, np.float32),
                                      np.ascontiguousarray(t_params, np.float32), B, s,
                                      np.ascontiguousarray(a_idx, np.int32), np.ascontiguousarray(r, np.float32),
                                      np.ascontiguousarray(s_next, np.float64).reshape(B, -1),
                                      np.ascontiguousarray(done, np.uint8),
                                      np.ascontiguousarray(mask3, np.uint8).reshape(B, 3), gamma, g, tgt,
                                      None if rin is None else rin.ctypes.data, dec.ctypes.data, mg.ctypes.data)
    return loss, g, dec, mg


# ---------------------------------------------------------------- deeper bf16 Q-net (configs[2])
def deep_nparams(bs: int, C: int) -> int:
    return int(lib().orc_deep_nparams(bs, C))


def deep_forward(bs: int, C: int, params: np.ndarray, x: np.ndarray) -> np.ndarray:
    """The configs[2] net with the device's bf16 rounding points, fp64 sums."""
    x = np.ascontiguousarray(x, np.float64).reshape(-1, C * bs * bs)
    B = x.shape[0]
    q = np.zeros((B, 3), np.float64)
    lib().orc_deep_forward(bs, C, np.ascontiguousarray(params, np.float32), B, x, q)
    return q


def deep_loss_grad(bs, C, q_params, t_params, s, a_idx, r, s_next, done, mask3, gamma=0.97):
    s = np.ascontiguousarray(s, np.float64).reshape(-1, C * bs * bs)
    B = s.shape[0]
    g = np.zeros(len(q_params), np.float64)
    tgt = np.zeros(B, np.float64)
    loss = lib().orc_deep_loss_grad(bs, C, np.ascontiguousarray(q_params, np.float32),
                                    np.ascontiguousarray(t_params, np.float32), B, s,
                                    np.ascontiguousarray(a_idx, np.int32), np.ascontiguousarray(r, np.float32),
                                    np.ascontiguousarray(s_next, np.float64).reshape(B, -1),
                                    np.ascontiguousarray(done, np.uint8),
                                    np.ascontiguousarray(mask3, np.uint8).reshape(B, 3), gamma, g, tgt)
    return loss, g, tgt


def rmsprop(theta, acc, grad, eta=5e-4, rho=0.9, eps=1e-8):
    theta = np.array(theta, np.float32, copy=True)
    acc = np.array(acc, np.float32, copy=True)
    lib().orc_rmsprop(len(theta), theta, acc, np.ascontiguousarray(grad, np.float32), eta, rho, eps)
    return theta, acc


# ---------------------------------------------------------------- Laplace
def welford_center(D: np.ndarray):
    """D: [K, P] (K snapshot columns of the reference's P x K matrix)."""
    D = np.array(D, np.float64, copy=True, order="C")
    K, P = D.shape
    mean = np.zeros(P, np.float64)
    var = np.zeros(P, np.float64)
    lib().orc_welford_center(P, K, D, mean, var)
    return D, mean, var


def gram(D: np.ndarray) -> np.ndarray:
    D = np.ascontiguousarray(D, np.float64)
    K, P = D.shape
    G = np.zeros((K, K), np.float64)
    lib().orc_gram(P, K, D, G)
    return G
