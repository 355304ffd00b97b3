"""CPU (gloo, world_size 2): the data-parallel host plumbing — RCCL unique-id
shipping, max-over-ranks timing, throughput aggregation — and the DP update
semantics the in-library RCCL all-reduce implements: the mean of per-rank
mean-loss gradients equals the gradient of the mean loss over the union batch
(equal shard sizes), checked with the oracle."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    import snake_amd.dist as sd
    ns = vars(sd)
    out = {}
    payload = bytes(range(128)) if rank == 0 else None
    out["uid"] = ns["broadcast_bytes"](dist, payload, rank)
    out["tmax"] = ns["max_over_ranks"](dist, 1.0 + rank)
    out["value"] = ns["aggregate_throughput"](4096, 10, world, out["tmax"])
    # DP gradient mean == union-batch gradient
    rng = np.random.default_rng(42)
    bs, C, B = 8, 2, 6
    P = oracle.qnet_nparams(bs, C)
    p = (rng.standard_normal(P) * 0.1).astype(np.float32)
    s = rng.integers(-1, 3, size=(world * B, C, bs * bs))
    sn = rng.integers(-1, 3, size=(world * B, C, bs * bs))
    a = rng.integers(0, 3, world * B)
    r = rng.standard_normal(world * B).astype(np.float32)
    d = rng.integers(0, 2, world * B).astype(np.uint8)
    m = rng.integers(0, 2, (world * B, 3)).astype(np.uint8)
    sl = slice(rank * B, (rank + 1) * B)
    _, g, _ = oracle.dqn_loss_grad(bs, C, p, p, s[sl], a[sl], r[sl], sn[sl], d[sl], m[sl])
    import torch
    gt = torch.from_numpy(g.copy())
    dist.all_reduce(gt)
    gt /= world
    _, gall, _ = oracle.dqn_loss_grad(bs, C, p, p, s, a, r, sn, d, m)
    out["dp_err"] = float(np.abs(gt.numpy() - gall).max() / np.abs(gall).max())
    q.put((rank, out))
    dist.destroy_process_group()


def test_dp_plumbing_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r]["uid"] == bytes(range(128))
        assert res[r]["tmax"] == 2.0
        assert res[r]["value"] == 2 * 4096 * 10 / 2.0
        assert res[r]["dp_err"] < 1e-12


def _gram_worker(rank, world, port, q):
    """One rank of the sharded D(50k) Gram: its tile list from the library
    (host-only snk_gram_tiles), the tiles' values taken from a reference Gram,
    gathered to rank 0 over gloo (the RCCL send/recv stand-in) and unpacked
    there the way gram_unpack_kernel does (lower tile + mirror)."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    import snake_amd as snk
    out = {}
    for n in (1000, 50_000 // 16):            # ragged last tile row (1000 = 7*128 + 104), and 3125
        rng = np.random.default_rng(n)
        J = rng.standard_normal((n, 40))
        Gref = J @ J.T
        tiles = snk.gram_tiles(n, rank, world)
        packed = np.zeros((len(tiles), 128, 128))
        for k, (i0, j0) in enumerate(tiles):
            blk = Gref[i0:i0 + 128, j0:j0 + 128]
            packed[k, :blk.shape[0], :blk.shape[1]] = blk
        objs = [None] * world
        dist.all_gather_object(objs, (tiles, packed))
        if rank == 0:
            G = np.full((n, n), np.nan)
            seen = set()
            for tl, pk in objs:
                for (i0, j0), blk in zip(tl, pk):
                    assert j0 <= i0 and (i0, j0) not in seen
                    seen.add((int(i0), int(j0)))
                    ii, jj = np.meshgrid(np.arange(i0, min(i0 + 128, n)), np.arange(j0, min(j0 + 128, n)),
                                         indexing="ij")
                    low = jj <= ii
                    G[ii[low], jj[low]] = blk[:ii.shape[0], :ii.shape[1]][low]
                    G[jj[low], ii[low]] = blk[:ii.shape[0], :ii.shape[1]][low]
            T = (n + 127) // 128
            out[n] = (len(seen) == T * (T + 1) // 2, bool(np.array_equal(G, Gref)),
                      [len({(int(i0) // 256, int(j0) // 256) for i0, j0 in tl}) for tl, _ in objs])
    q.put((rank, out))
    dist.destroy_process_group()


def test_gram_shards_gloo_world2_and_4():
    """D(50k) across ranks: the tile shards of every rank are disjoint, cover
    the lower triangle exactly once, are balanced to within one of the K-split
    Gram's 256 x 256 tiles (its unit of work: shards are runs of that tile order,
    cut at the nearest tile; gram_tiles lists each one's 128 x 128 subtiles), and
    reassemble (with the mirror) to the full Gram."""
    for world in (2, 4):
        port = _free_port()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_gram_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=240) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for n, (covered, equal, counts) in res[0].items():
            assert covered and equal, (world, n)
            assert max(counts) - min(counts) <= 1, counts
