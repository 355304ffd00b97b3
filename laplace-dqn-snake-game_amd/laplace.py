"""Laplace D build (compute_D.jl, la_utils.jl:14-36, plot_traj.jl:10-16) and
the per-sample-Jacobian Gram of the north star, on the GPU.

`LaplaceD` owns the reference's `deviation_matrix` (P x K Float64; stored
column by column, i.e. Julia's own memory order) together with the Welford
`MeanStd` state. `compute_D(tr)` drives a `Trainer` through the reference's
schedule: burn-in, one snapshot every `thin` updates, Welford + centring
once K columns are in.
"""
from __future__ import annotations

import ctypes as C
import math
import warnings

import numpy as np

from . import _lib
from ._lib import DeviceArray, call, vp
from .qnet import DQNModel
from .replay import ReplayBuffer


class LaplaceD:
    """`deviation_matrix = zeros(Float64, (param_count, K))` + `MeanStd(param_count)`
    (compute_D.jl:50-55)."""

    def __init__(self, n_params: int, K: int = 1000):
        self.P, self.K = int(n_params), int(K)
        h = vp()
        call("snk_laplace_create", C.byref(h), self.P, self.K)
        self._h = h
        self.fitted = False

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.snk_laplace_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def snapshot(self, model: DQNModel, pos: int) -> None:
        """compute_D.jl:69-70 `deviation_matrix[:, position] = Float64.(theta)` (pos 0-based)."""
        call("snk_laplace_snapshot", self._h, model.handle, int(pos))

    def set_column(self, pos: int, col) -> None:
        col = np.ascontiguousarray(col, np.float64)
        assert col.size == self.P, (col.size, self.P)
        call("snk_laplace_set_column", self._h, int(pos), _lib.ptr(col))

    def fit_center(self) -> None:
        """compute_D.jl:74-81: `for c in eachcol(D) fit!(o, c) end; D .-= mean(o)`."""
        call("snk_laplace_fit_center", self._h)
        self.fitted = True

    def _get(self, which: int, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        call("snk_laplace_get", self._h, which, _lib.ptr(out), out.nbytes)
        return out

    def D(self) -> np.ndarray:
        """[K, P]: row k is column k of the reference's P x K matrix."""
        return self._get(_lib.SNK_LAP_D, (self.K, self.P), np.float64)

    def mean(self) -> np.ndarray:
        """compute_D.jl:29 `mean(o::MeanStd)`."""
        return self._get(_lib.SNK_LAP_MEAN, self.P, np.float64)

    def var(self) -> np.ndarray:
        """compute_D.jl:30 `var(o) = m2 ./ max(n - 1, 1)`."""
        return self._get(_lib.SNK_LAP_VAR, self.P, np.float64)

    def std(self) -> np.ndarray:
        """compute_D.jl:31 (sqrt of the device var)."""
        return np.sqrt(self.var())

    def gram(self) -> tuple[np.ndarray, float]:
        """G = D'D (K x K, fp64 result of fp32 MFMA with fp64 accumulation) and the Gram kernel's ms."""
        ms = C.c_float(0.0)
        call("snk_laplace_gram", self._h, C.byref(ms))
        return self._get(_lib.SNK_LAP_GRAM, (self.K, self.K), np.float64), ms.value

    def eig(self, G: np.ndarray | None = None):
        """Eigen-decomposition of the device Gram D'D: (lambda, V) with
        lambda = S.^2/(K-1) in svd order (descending) and V the right singular
        vectors of D (plot_traj.jl:10-16: U, S, V = svd(D))."""
        if G is None:
            G, _ = self.gram()
        w, V = np.linalg.eigh(G)
        order = np.argsort(w)[::-1]
        w = np.clip(w[order], 0.0, None)
        return w / (self.K - 1), V[:, order]

    @staticmethod
    def n_cols(lam: np.ndarray, frac: float = 0.99) -> int:
        """plot_traj.jl:47-63 compute_n_cols: how many leading eigenvalues of
        D'D/(K-1) (svd order) account for 99 % of their sum."""
        lim = frac * float(np.sum(lam))
        cum, n = 0.0, 0
        for v in lam:
            cum += float(v)
            n += 1
            if cum >= lim:
                break
        return n

    def trajectory_2d(self, G: np.ndarray | None = None) -> np.ndarray:
        """plot_traj.jl:65-67 Y = U[:, 1:2]' * D: the K snapshots projected on
        the two leading directions, [2, K]. With D = U S V', U[:, i]' D = S_i V[:, i]',
        so it follows from the Gram alone."""
        lam, V = self.eig(G)
        S = np.sqrt(lam[:2] * (self.K - 1))
        return S[:, None] * V[:, :2].T

    def spectrum(self, G: np.ndarray | None = None, floor: float = 1e-7) -> np.ndarray:
        """plot_traj.jl:10-19: lambda = S.^2/(K-1) of svd(D), the eigenvalues of
        D'D/(K-1), keeping those > 1e-7 (host analysis of the device Gram,
        as plot_traj.jl is analysis of the saved D)."""
        if G is None:
            G, _ = self.gram()
        lam = np.linalg.eigvalsh(G) / (self.K - 1)
        return np.sort(lam[lam > floor])[::-1]


def compute_D(tr, K: int = 1000, thin: int = 10, burn_in: int = 50_000, graph: bool = True,
              reset_optimizer: bool = True, schedule: str = "episode", n_batches: int | None = None,
              on_update=None, strict: bool = False) -> LaplaceD | None:
    """compute_D.jl:33-86 on a Trainer: fill_buffer!, a fresh RMSProp state
    (`Flux.setup`, :47), then the training loop `while nb <= n_batches`
    (:56-58, nb from 1, n_batches = tr.n_batches unless given): from
    nb == burn_in on (:61), at nb % thin == 0 the current q_net goes into the
    next column *before* that nb's update runs (:67-71); right after the K-th
    column (no update at that nb): Welford + centring (:74-81) and return (the
    BSON save of :84 is the caller's business). update_target_net! runs after
    update nb when nb % rate == 0 (:129-132).

    If the loop ends (nb > n_batches) before the K-th column, the reference
    returns `nothing` without building D; so does this: the updates still run,
    a RuntimeWarning names the nb the K-th column needs, and None is returned
    (strict=True raises ValueError instead).

    schedule="episode": the reference's loop body, one full epsilon-greedy
    episode stored and one B-sample update per nb (:89-138, EpisodeLoop).
    schedule="batched": one lockstep step of tr's n_envs games per update
    (the device trainer, graph-replayed), with the same nb bookkeeping.

    on_update(nb, loss): observer called after every update (episode schedule;
    loss = that update's Huber loss) or after every run of updates ending at nb
    (batched schedule; loss = None). Test infrastructure uses it to check each
    update against the oracle."""
    from .trainer import EpisodeLoop, fill_buffer_

    model = tr.model
    n_batches = int(tr.n_batches if n_batches is None else n_batches)
    lap = LaplaceD(model.P, K)
    first = burn_in if burn_in % thin == 0 else burn_in + (thin - burn_in % thin)   # first nb snapshotted
    snaps = [first + pos * thin for pos in range(K)]        # nb at which column pos is taken
    if schedule == "episode":
        loop = EpisodeLoop(tr)
        loop.fill()
    elif schedule == "batched":
        if tr.updates_per_iter != 1:
            raise ValueError("compute_D snapshots between single updates: use updates_per_iter = 1")
        fill_buffer_(tr, graph=graph)
        tr.set_nb(1)
    else:
        raise ValueError(f"unknown schedule {schedule!r}")
    if reset_optimizer:
        model.set_params(np.zeros(model.P, np.float32), _lib.SNK_NET_OPT_STATE)

    def updates(nb_from: int, nb_to: int) -> None:          # updates nb_from .. nb_to (inclusive)
        if nb_to < nb_from:
            return
        if schedule == "episode":
            for nb in range(nb_from, nb_to + 1):
                _, loss = loop.step(nb)
                if on_update is not None:
                    on_update(nb, loss)
        else:
            tr.run(nb_to - nb_from + 1, learn=True, graph=graph)
            if on_update is not None:
                on_update(nb_to, None)

    nb = 1
    for pos, at in enumerate(snaps):
        if at > n_batches:                                  # `while nb <= n_batches` ends first
            updates(nb, n_batches)
            msg = (f"compute_D: the loop ended at nb = {n_batches} (n_batches) before the K-th snapshot "
                   f"(column {pos + 1} of {K} falls at nb = {at}); returning None as compute_D.jl:58 "
                   f"returns nothing. Raise n_batches to >= {snaps[-1]} to build D.")
            if strict:
                raise ValueError(msg)
            warnings.warn(msg, RuntimeWarning, stacklevel=2)
            return None
        updates(nb, at - 1)
        nb = at
        lap.snapshot(model, pos)
    lap.fit_center()
    return lap


def jacobian(model: DQNModel, buf: ReplayBuffer, n: int | None = None, slots=None) -> np.ndarray:
    """Per-sample Jacobians J[s] = dQ(state_s)[a_s]/dtheta (Flux.destructure
    order) for replay slots `slots` (default 0..n-1): [n, P] float32."""
    if slots is not None:
        slots = np.ascontiguousarray(slots, np.int64)
        n = slots.size
        dslots = DeviceArray.from_host(slots)
    else:
        dslots = None
    n = int(n if n is not None else len(buf))
    J = DeviceArray((n, model.P), np.float32)
    call("snk_jacobian", model.handle, buf.handle, dslots.ptr if dslots is not None else None, n, J.ptr)
    return J.numpy()


def jacobian_gram(model: DQNModel, buf: ReplayBuffer, n: int | None = None, *, out: DeviceArray | None = None,
                  host: bool = True):
    """G = J J' over replay slots 0..n-1 (default: the whole buffer).
    Returns (G, ms) with G a host [n, n] float32 array (or the DeviceArray
    when host=False) and ms the 4 phase times (forward + data gradients,
    per-sample conv Jacobians, conv Gram, dense terms + mirror)."""
    n = int(n if n is not None else len(buf))
    G = out if out is not None else DeviceArray((n, n), np.float32)
    ms = (C.c_float * 4)()
    call("snk_jacobian_gram", model.handle, buf.handle, n, G.ptr, ms)
    t = [float(v) for v in ms]
    return (G.numpy() if host else G), t


def gram_tiles(n: int, rank: int = 0, nranks: int = 1) -> np.ndarray:
    """The 128 x 128 lower-triangle tiles of the n x n Gram that shard
    rank / nranks computes: [count, 2] top-left (row, col) elements, a
    contiguous run of the XCD-aware supertile order (host only)."""
    cnt = C.c_int64(0)
    call("snk_gram_tiles", int(n), int(rank), int(nranks), None, C.byref(cnt))
    out = np.zeros((cnt.value, 2), np.int32)
    call("snk_gram_tiles", int(n), int(rank), int(nranks), _lib.ptr(out), C.byref(cnt))
    return out


def jacobian_gram_shard(model: DQNModel, buf: ReplayBuffer, n: int, rank: int, nranks: int,
                        out: DeviceArray) -> list:
    """This rank's tiles (and their mirror) of G = J J' over slots 0..n-1
    written into `out` (a device [n, n] float32 array; other entries are left
    as they are). Returns the 4 phase times (ms)."""
    ms = (C.c_float * 4)()
    call("snk_jacobian_gram_shard", model.handle, buf.handle, int(n), int(rank), int(nranks), out.ptr, ms)
    return [float(v) for v in ms]


def jacobian_gram_gather(comm, n: int, out: DeviceArray, root: int = 0) -> None:
    """Collective: every rank's shard tiles onto root's `out` (RCCL send/recv)."""
    call("snk_jacobian_gram_gather", comm.handle, int(n), out.ptr, int(root))


def d_build_seconds(ms) -> float:
    """Wall time of one Jacobian-Gram D build from its phase times."""
    return sum(ms) / 1e3 if ms else math.nan


# ---------------------------------------------------------------- Laplace sampling
def laplace_normals(seed: int, model: int, which: int, i0: int, n: int) -> np.ndarray:
    """The counter-based N(0, 1) stream behind sample_model: z1 (which=1,
    indexed by Flux parameter index) or z2 (which=2, indexed by column k)
    of model `model`."""
    out = np.empty(int(n), np.float64)
    call("snk_laplace_normals", int(seed), int(model), int(which), int(i0), int(n), _lib.ptr(out))
    return out


def sample_model(lap: LaplaceD, model: DQNModel, n: int = 0, seed: int = 0) -> np.ndarray:
    """la_utils.jl:83-95 `sample_model(mean, var, D, re)` for sample n:
    w = mean + 1/sqrt(2) * sqrt.(Diagonal(|var|)) * z1 + 1/sqrt(2(K-1)) * D * z2,
    computed on the device in Float64 term by term, returned as Float32 in
    Flux.destructure order (what `re(w)` holds). `lap` must be fitted
    (mean, var and the centred D, la_utils.jl:161-167)."""
    if not lap.fitted:
        raise RuntimeError("LaplaceD.fit_center() first: sample_model needs mean, var and the centred D")
    out = np.empty(model.P, np.float32)
    call("snk_laplace_sample_params", lap.handle, model.handle, int(seed), int(n), _lib.ptr(out))
    return out


def laplace_sampling_(tr, lap: LaplaceD, n_models: int = 5000, epsilon: float = 0.0, *, seed: int = 0,
                      chunk: int = 0) -> dict:
    """la_utils.jl:97-118 `laplace_sampling!(tr, mean, var, D; n_models=5000)`:
    the greedy episode reward of tr.model, then n_models sampled models each
    play one greedy episode (all in lockstep on the device); the transitions
    of every model whose episode reward beats tr.model's are stored into
    tr.buffer in model order. `epsilon` is accepted for the reference's
    signature; like the reference (`play_episode(model, 0.0f0)`, :105) the
    sampled models play greedily. Returns n_better_models, the reference
    reward and every model's (reward, length)."""
    del epsilon
    if not lap.fitted:
        raise RuntimeError("LaplaceD.fit_center() first")
    n_models = int(n_models)
    rew = np.zeros(max(n_models, 1), np.float32)
    length = np.zeros(max(n_models, 1), np.int32)
    trr, nb = C.c_float(0), C.c_int64(0)
    call("snk_laplace_sampling", lap.handle, tr.model.handle, tr.buffer.handle, n_models, int(seed), int(chunk),
         C.byref(trr), C.byref(nb), _lib.ptr(rew), _lib.ptr(length))
    return {"n_better_models": nb.value, "tr_reward": float(trr.value), "rewards": rew[:n_models],
            "lengths": length[:n_models]}
