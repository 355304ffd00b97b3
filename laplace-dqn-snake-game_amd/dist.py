"""Data-parallel replicas over RCCL (one process per GPU).

The reference is single-process; this is new. Envs shard by
rank (each rank steps its own n_envs, no env exchange: weak scaling); each
DQN update all-reduces (mean) the gradient inside libsnakehip (RCCL over
xGMI) so the replicas stay identical. The host side only ships RCCL's
128-byte unique id from rank 0 to the others over torch.distributed (gloo),
and reduces the timing scalars.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import call, vp


def broadcast_bytes(dist, payload: bytes | None, rank: int, src: int = 0, size: int = 128) -> bytes:
    """Ship `size` bytes from rank `src` to every rank over a (gloo) group."""
    import torch
    t = torch.zeros(size, dtype=torch.uint8)
    if rank == src:
        assert payload is not None and len(payload) == size
        t.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
    dist.broadcast(t, src)
    return bytes(t.tolist())


def max_over_ranks(dist, value: float) -> float:
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_throughput(n_envs_per_rank: int, steps: int, world: int, max_elapsed: float) -> float:
    """bench.py contract: env-steps of ALL ranks / max-over-ranks wall time."""
    return world * n_envs_per_rank * steps / max_elapsed


class Comm:
    """An RCCL communicator owned by libsnakehip."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = vp()
        call("snk_comm_create", C.byref(h), nranks, rank, buf)
        self._h = h
        self.nranks, self.rank = nranks, rank

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        call("snk_comm_unique_id", buf)
        return bytes(buf)

    @property
    def handle(self):
        return self._h

    def info(self) -> tuple[int, int]:
        """(ranks, rank) as RCCL reports them for this communicator (ncclCommCount,
        ncclCommUserRank)."""
        n, r = C.c_int32(0), C.c_int32(0)
        call("snk_comm_info", self._h, C.byref(n), C.byref(r))
        return n.value, r.value

    def allreduce_mean(self, dev_ptr: int, n: int) -> None:
        call("snk_comm_allreduce_mean", self._h, vp(dev_ptr), n)

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.snk_comm_destroy(self._h)
            self._h = None


def dist_attach(trainer, dist, rank: int, world: int) -> Comm:
    """Join `trainer` to a data-parallel group: RCCL communicator from a unique
    id made on rank 0, q_net broadcast from rank 0, per-update gradient mean."""
    uid = Comm.unique_id() if rank == 0 else None
    uid = broadcast_bytes(dist, uid, rank)
    comm = Comm(world, rank, uid)
    call("snk_trainer_set_comm", trainer.handle, comm.handle)
    trainer._comm = comm
    return comm


def dist_detach(trainer) -> None:
    """Leave the data-parallel group: later updates stay local (no collective),
    so one rank can keep training (e.g. rank 0's D builds after a timed
    multi-GPU run) while the others exit."""
    call("snk_trainer_set_comm", trainer.handle, None)
    trainer._comm = None
