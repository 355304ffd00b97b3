"""ReplayBuffer on the GPU (structs.jl:104-116, utils.jl:262-383).

The ring holds, per transition, the n_frames+1 boards b_{t-C}..b_t and the
metadata of the reference's `Experience` tuple (imports.jl:27-36): action
index into available_actions, reward, done, the next state's suicidal mask,
and the directions from which `av_actions` / `av_next_actions` follow.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import DeviceArray, call, ptr, vp
from .env import ALL_ACTIONS, NULL_ACTION, available_action_codes


class ReplayBuffer:
    """structs.jl:110 `ReplayBuffer(capacity=50000)` with `batch_size = 64`."""

    def __init__(self, capacity: int = 50000, *, board_size: int = 10, n_frames: int = 2,
                 batch_size: int = 64):
        self.capacity = int(capacity)
        self.batch_size = int(batch_size)
        self.board_size = int(board_size)
        self.n_frames = int(n_frames)
        h = vp()
        call("snk_replay_create", C.byref(h), self.capacity, self.board_size, self.n_frames,
             self.batch_size)
        self._h = h
        self._idx = DeviceArray(self.batch_size, np.int64)

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.snk_replay_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def __len__(self) -> int:  # Base.length(rpb) (utils.jl:265)
        n = C.c_int64(0)
        call("snk_replay_length", self._h, C.byref(n))
        return n.value

    @property
    def count(self) -> int:
        n = C.c_int64(0)
        call("snk_replay_position", self._h, C.byref(n))
        return n.value

    @property
    def position(self) -> int:
        """The reference's 1-based `rpb.position` (utils.jl:267-277): 1 while
        filling, then the next slot to overwrite."""
        c = self.count
        return 1 if c < self.capacity else (c - self.capacity) % self.capacity + 1


def store_(rpb: ReplayBuffer, frames, act_idx, reward, done, mask, dirs) -> None:
    """store! (utils.jl:267-277) of B explicit transitions.

    frames [B, C+1, bs*bs] int8 (b_{t-C}..b_t, column-major cells); act_idx
    index into available_actions; mask [B, 3] or packed bits; dirs packed
    prev_dir | dir<<2 | lost<<4."""
    frames = np.ascontiguousarray(frames, np.int8)
    B = frames.shape[0]
    mask = np.asarray(mask)
    if mask.ndim == 2:
        mask = (mask[:, 0].astype(np.uint8) | (mask[:, 1].astype(np.uint8) << 1)
                | (mask[:, 2].astype(np.uint8) << 2))
    call("snk_replay_store", rpb._h, B, ptr(frames), ptr(np.ascontiguousarray(act_idx, np.uint8)),
         ptr(np.ascontiguousarray(reward, np.float32)), ptr(np.ascontiguousarray(done, np.uint8)),
         ptr(np.ascontiguousarray(mask, np.uint8)), ptr(np.ascontiguousarray(dirs, np.uint8)))


def isready(rpb: ReplayBuffer) -> bool:  # utils.jl:293-296
    return len(rpb) >= rpb.batch_size


def isfull(rpb: ReplayBuffer) -> bool:  # utils.jl:289-291 (position == capacity)
    return rpb.position == rpb.capacity


def empty_buffer_(rpb: ReplayBuffer) -> None:  # utils.jl:311-314
    call("snk_replay_empty", rpb._h)


def sample(rpb: ReplayBuffer, seed: int = 0, draw: int = 0):
    """utils.jl:280-287: min(batch_size, length) distinct slot indices, drawn
    on the device. Returns (DeviceArray of int64 indices, B)."""
    B = C.c_int32(0)
    call("snk_replay_sample", rpb._h, seed, draw, rpb._idx.ptr, C.byref(B))
    return rpb._idx, B.value


def stack_exp(rpb: ReplayBuffer, idx, B: int | None = None) -> dict:
    """utils.jl:343-383 for the slots `idx` (host array or DeviceArray).

    Returns host arrays: states / next_states Float32 (bs,bs,C,B) Julia memory
    as [B, C, bs*bs]; actions 1-based Int32; rewards Float32; dones Bool;
    suicidal_mask [B, 3] Bool; av_actions / a_array / av_next_actions as
    direction tuples."""
    if isinstance(idx, DeviceArray):
        d_idx = idx
        B = int(B if B is not None else idx.shape[0])
    else:
        idx = np.ascontiguousarray(idx, np.int64)
        B = len(idx)
        d_idx = DeviceArray.from_host(idx)
    bs, nf = rpb.board_size, rpb.n_frames
    st = DeviceArray((B, nf, bs * bs), np.float32)
    nst = DeviceArray((B, nf, bs * bs), np.float32)
    act = DeviceArray(B, np.int32)
    rew = DeviceArray(B, np.float32)
    done = DeviceArray(B, np.uint8)
    mask = DeviceArray((B, 3), np.uint8)
    dirs = DeviceArray(B, np.uint8)
    call("snk_replay_gather", rpb._h, d_idx.ptr, B, st.ptr, act.ptr, rew.ptr, nst.ptr, done.ptr,
         mask.ptr, dirs.ptr)
    d = dirs.numpy()
    av = [[ALL_ACTIONS[a] for a in available_action_codes(x & 3)] for x in d]
    av_next = [([NULL_ACTION] * 3 if (x >> 4) & 1 else
                [ALL_ACTIONS[a] for a in available_action_codes((x >> 2) & 3)]) for x in d]
    a_array = [ALL_ACTIONS[(x >> 2) & 3] for x in d]
    return dict(states=st.numpy(), actions=act.numpy(), rewards=rew.numpy(), next_states=nst.numpy(),
                dones=done.numpy().astype(bool), av_actions=av, a_array=a_array,
                suicidal_mask=mask.numpy().astype(bool), av_next_actions=av_next, dirs=d)
