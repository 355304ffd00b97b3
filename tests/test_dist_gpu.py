"""GPU: the in-library RCCL path on one device (a 1-rank communicator). The
averaged gradient of one rank is the gradient itself, so a DP trainer must
match the plain trainer bit for bit — eager and hipGraph-captured."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _train(snk, comm_graph):
    tr = snk.Trainer(n_batches=20, target_update_rate=8, n_envs=96, board_size=12, n_frames=2, capacity=600,
                     decay=1e-3, seed=5)
    if comm_graph is not None:
        uid = snk.Comm.unique_id()
        comm = snk.Comm(1, 0, uid)
        snk._lib.call("snk_trainer_set_comm", tr.handle, comm.handle)
        tr._comm = comm
        snk.train_(tr, graph=comm_graph)
    else:
        snk.train_(tr, graph=True)
    return tr.model.get_params(), tr.losses


def test_rccl_single_rank_matches_plain(snk):
    p0, l0 = _train(snk, None)
    p1, l1 = _train(snk, False)
    assert np.array_equal(p0, p1) and np.array_equal(l0, l1)
    p2, l2 = _train(snk, True)
    assert np.array_equal(p0, p2) and np.array_equal(l0, l2)


def test_comm_allreduce_and_broadcast(snk):
    comm = snk.Comm(1, 0, snk.Comm.unique_id())
    x = np.arange(1000, dtype=np.float32)
    d = snk.DeviceArray.from_host(x)
    comm.allreduce_mean(d.ptr.value, 1000)
    snk._lib.call("snk_comm_broadcast", comm.handle, d.ptr, 1000, 0)
    snk._lib.call("snk_synchronize")
    assert np.array_equal(d.numpy(), x)


def test_detach_then_train_locally(snk):
    """dist_detach (bench.py before rank 0's single-GPU extras): a trainer that
    leaves its communicator keeps training with local updates and its
    recaptured graphs; a 1-rank run detached half way matches the plain run."""
    def run(detach):
        tr = snk.Trainer(n_batches=20, target_update_rate=8, n_envs=96, board_size=12, n_frames=2, capacity=600,
                         decay=1e-3, seed=5)
        if detach:
            comm = snk.Comm(1, 0, snk.Comm.unique_id())
            snk._lib.call("snk_trainer_set_comm", tr.handle, comm.handle)
            tr._comm = comm
        snk.fill_buffer_(tr)
        tr.run(10, learn=True, graph=True)
        if detach:
            snk.dist_detach(tr)
            assert tr._comm is None
        tr.run(10, learn=True, graph=True)
        return tr.model.get_params(), tr.losses
    p0, l0 = run(False)
    p1, l1 = run(True)
    assert np.array_equal(p0, p1) and np.array_equal(l0, l1)
