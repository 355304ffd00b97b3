"""Trainer, train!, fill_buffer!, epsilon_greedy and play_episode
(structs.jl:151-175, utils.jl:153-259, 389-494) on the GPU.

The batched trainer keeps the reference's per-update schedule — epsilon
decays by `decay` per update, update_target_net! when nb % rate == 0
(nb = 0 included), n_batches + 1 updates in all — but feeds the replay from
`n_envs` games stepped in lockstep (`updates_per_iter` updates per lockstep
step) instead of one full episode per update. `train_(tr,
schedule="episode")` runs the reference's own loop instead (one whole
epsilon-greedy episode, stored, then one 64-sample update, utils.jl:434-482),
host-driven over the same device primitives.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import DeviceArray, call, vp
from .env import SnakeGame, step_indices_dev
from .qnet import DQNModel
from .replay import ReplayBuffer, sample, stack_exp


def epsilon_greedy(game: SnakeGame, model: DQNModel, epsilon: float, *, seed: int = 0,
                   act: DeviceArray | None = None) -> np.ndarray:
    """utils.jl:153-172 for every env: action indices into available_actions."""
    act = act if act is not None else DeviceArray(game.n_envs, np.uint8)
    call("snk_dqn_act", model.handle, game.handle, float(epsilon), int(seed), act.ptr)
    return act.numpy()


class Trainer:
    """structs.jl:164 `Trainer(; n_batches=1000, target_update_rate=1000,
    epsilon=1.0, epsilon_end=0.05, decay=1e-6, save=true, game, model)`."""

    def __init__(self, *, n_batches: int = 1000, target_update_rate: int = 1000, epsilon: float = 1.0,
                 epsilon_end: float = 0.05, decay: float = 1e-6, save: bool = False, game: SnakeGame | None = None,
                 model: DQNModel | None = None, n_envs: int = 1, board_size: int = 10, n_frames: int = 2,
                 capacity: int = 50000, batch_size: int = 64, updates_per_iter: int = 1, gamma: float = 0.97,
                 seed: int = 1234, loss_log_capacity: int = 1 << 20, graph_unroll: int = 0, deep: bool = False):
        self.game = game if game is not None else SnakeGame(board_size, n_frames, n_envs=n_envs, autoreset=True)
        if not self.game.autoreset:
            raise ValueError("the batched trainer needs auto-reset games")
        bs, nf = self.game.board_size, self.game.n_frames
        self.model = model if model is not None else DQNModel(bs, 3, n_frames=nf, seed=seed, deep=deep)
        self.buffer = ReplayBuffer(capacity, board_size=bs, n_frames=nf, batch_size=batch_size)
        self.n_batches, self.target_update_rate = int(n_batches), int(target_update_rate)
        self.epsilon, self.epsilon_end, self.decay = float(epsilon), float(epsilon_end), float(decay)
        self.save, self.gamma, self.seed = bool(save), float(gamma), int(seed)
        self.updates_per_iter = int(updates_per_iter)
        self.loss_log_capacity = int(loss_log_capacity)
        # schedule="episode" history (tr.episode_rewards / tr.losses of utils.jl:477-478)
        self.episode_rewards: list[float] = []
        self.episode_losses: list[float] = []
        cfg = _lib.TrainerCfg(self.epsilon, self.epsilon_end, self.decay, self.updates_per_iter,
                              self.target_update_rate, self.gamma, self.seed, self.loss_log_capacity,
                              int(graph_unroll))
        h = vp()
        call("snk_trainer_create", C.byref(h), self.game.handle, self.model.handle, self.buffer.handle,
             C.byref(cfg))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.snk_trainer_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def run(self, iters: int, learn: bool = True, graph: bool = True) -> None:
        call("snk_trainer_run", self._h, int(iters), int(learn), int(graph))

    def run_partial(self, n_updates: int) -> None:
        """One lockstep iteration with n_updates (< updates_per_iter) updates."""
        call("snk_trainer_run_partial", self._h, int(n_updates))

    def set_nb(self, nb: int) -> None:
        """The reference's batch counter for update_target_net! (nb % rate == 0,
        then nb += 1): train! starts at 0 (utils.jl:431), compute_D at 1
        (compute_D.jl:56)."""
        call("snk_trainer_set_nb", self._h, int(nb))

    def set_trace(self, ring: DeviceArray | None) -> None:
        """Copy every update's finished gradient into ring[slot] (a device
        [slots, P] float32 array; slot = position of the update in the run's
        launch sequence % slots); None turns it off. Test infrastructure: it
        makes each update of a captured multi-iteration graph observable."""
        if ring is None:
            call("snk_trainer_set_trace", self._h, None, 0)
        else:
            if ring.dtype != np.float32 or len(ring.shape) != 2 or ring.shape[1] != self.model.P:
                raise ValueError(f"gradient trace ring must be float32 [slots, {self.model.P}], got "
                                 f"{ring.dtype} {ring.shape}")
            call("snk_trainer_set_trace", self._h, ring.ptr, int(ring.shape[0]))
        self._trace = ring

    def set_act_trace(self, acts: DeviceArray | None, q: DeviceArray | None = None) -> None:
        """Copy every iteration's actions into acts[slot] (device [slots, n_envs]
        uint8) and, if given, its act-forward Q values into q[slot] (device
        [slots, n_envs, 3] float32); slot = iteration within the run's launch
        sequence % slots. Test infrastructure, as set_trace."""
        if acts is None:
            call("snk_trainer_set_act_trace", self._h, None, None, 0)
        else:
            # the library copies n_envs bytes (and n_envs x 3 floats) per slot inside the
            # captured graphs: a smaller ring would be written out of bounds
            if acts.dtype != np.uint8 or len(acts.shape) != 2 or acts.shape[1] != self.game.n_envs:
                raise ValueError(f"act trace ring must be uint8 [slots, {self.game.n_envs}], got {acts.dtype} {acts.shape}")
            if q is not None and (q.dtype != np.float32 or tuple(q.shape[1:]) != (self.game.n_envs, 3)):
                raise ValueError(f"Q trace ring must be float32 [slots, {self.game.n_envs}, 3], got {q.dtype} {q.shape}")
            if q is not None and q.shape[0] != acts.shape[0]:
                raise ValueError("act and Q trace rings need the same slot count")
            call("snk_trainer_set_act_trace", self._h, acts.ptr, q.ptr if q is not None else None,
                 int(acts.shape[0]))
        self._act_trace = (acts, q)

    def stats(self) -> dict:
        st = _lib.TrainerStats()
        call("snk_trainer_stats", self._h, C.byref(st))
        return {k: getattr(st, k) for k, _ in st._fields_ if k != "struct_size"}

    @property
    def losses(self) -> np.ndarray:
        """tr.losses (utils.jl:404-406), newest last (up to the log capacity)."""
        n = min(self.stats()["updates"], self.loss_log_capacity)
        out = np.zeros(self.loss_log_capacity, np.float64)
        call("snk_trainer_losses", self._h, _lib.ptr(out), self.loss_log_capacity)
        u = self.stats()["updates"]
        if u <= self.loss_log_capacity:
            return out[:n]
        k = u % self.loss_log_capacity
        return np.concatenate([out[k:], out[:k]])


def fill_buffer_(tr: Trainer, graph: bool = True) -> None:
    """utils.jl:389-402: play (with tr.epsilon) until more than `capacity`
    experiences have been stored."""
    need = tr.buffer.capacity + 1 - tr.buffer.count
    if need > 0:
        tr.run(math.ceil(need / tr.game.n_envs), learn=False, graph=graph)


def _episode_into(tr: "Trainer", game: SnakeGame, act: DeviceArray, epsilon: float, seed: int,
                  max_steps: int = 100000) -> tuple[int, float]:
    """play_episode (utils.jl:198-259) with the live q_net, every transition
    stored into tr.buffer as it happens (store!, utils.jl:267-277).
    Returns (steps, episode reward summed in Float32 as utils.jl:247)."""
    L, ep = 0, np.float32(0)
    while L < max_steps:
        call("snk_dqn_act", tr.model.handle, game.handle, float(epsilon), int(seed), act.ptr)
        step_indices_dev(game, act.ptr, replay=tr.buffer)
        o = game.last("reward", "done")
        ep = np.float32(ep + np.float32(o["reward"][0]))
        L += 1
        if o["done"][0]:
            break
    return L, float(ep)


class EpisodeLoop:
    """The reference's one-episode-per-update loop body, host-driven over the
    device primitives: one SnakeGame, tr.buffer, tr.model. Shared by train!
    (utils.jl:420-482, nb from 0) and compute_D (compute_D.jl:89-138, nb from 1).
    The replay draw of update u is `sample(seed, draw=u)` with u counting
    this loop's updates."""

    def __init__(self, tr: "Trainer"):
        self.tr = tr
        self.game = SnakeGame(tr.game.board_size, tr.game.n_frames, n_envs=1, autoreset=True)
        self.act = DeviceArray(1, np.uint8)
        self.eps = np.float32(tr.epsilon)
        self.draws = 0

    def fill(self) -> int:
        """fill_buffer! (utils.jl:389-402): play until more than capacity
        transitions were played."""
        tr, played = self.tr, 0
        while played <= tr.buffer.capacity:
            L, _ = _episode_into(tr, self.game, self.act, float(self.eps), tr.seed)
            played += L
        return played

    def step(self, nb: int) -> tuple[float, float]:
        """One episode into the buffer, one B-sample update (sample -> t_net
        target -> Huber -> backward -> RMSProp), update_target_net! when
        nb % rate == 0, epsilon decay (utils.jl:480). Returns (episode reward, loss)."""
        tr = self.tr
        _, ep_reward = _episode_into(tr, self.game, self.act, float(self.eps), tr.seed)
        idx, B = sample(tr.buffer, seed=tr.seed, draw=self.draws)
        self.draws += 1
        loss = tr.model.update(tr.buffer, idx, B, tr.gamma)
        if nb % tr.target_update_rate == 0:
            call("snk_dqn_sync_target", tr.model.handle)
        self.eps = max(np.float32(self.eps - np.float32(tr.decay)), np.float32(tr.epsilon_end))
        tr.epsilon = float(self.eps)
        return ep_reward, loss


def _train_episodes(tr: "Trainer") -> dict:
    """utils.jl:389-402 (fill_buffer!) and 420-482 (train!'s loop), one env:
    fill until more than `capacity` experiences were played; then for
    nb = 0..n_batches one EpisodeLoop.step."""
    loop = EpisodeLoop(tr)
    loop.fill()
    for nb in range(tr.n_batches + 1):                        # utils.jl:435 (nb <= n_batches)
        ep_reward, loss = loop.step(nb)
        tr.episode_rewards.append(ep_reward)
        tr.episode_losses.append(loss)
    return {"updates": tr.n_batches + 1, "episodes": len(tr.episode_rewards), "epsilon": float(loop.eps),
            "buffer_length": len(tr.buffer)}


def train_(tr: Trainer, trainer_name: str | None = None, graph: bool = True, schedule: str = "batched") -> dict:
    """utils.jl:420-494: fill the buffer, then n_batches + 1 DQN updates.
    schedule="batched": the lockstep device loop (snk_trainer_run);
    schedule="episode": the reference's one-episode-per-update loop."""
    if schedule == "episode":
        return _train_episodes(tr)
    if schedule != "batched":
        raise ValueError(f"unknown schedule {schedule!r}")
    fill_buffer_(tr, graph=graph)
    if tr.updates_per_iter > 0:
        total = tr.n_batches + 1 - tr.stats()["updates"]
        if total > 0:
            # exactly n_batches + 1 updates: full iterations, then one partial one
            full, rest = divmod(total, tr.updates_per_iter)
            tr.run(full, learn=True, graph=graph)
            if rest:
                tr.run_partial(rest)
    return tr.stats()


def play_episode(model: DQNModel, epsilon: float, *, actions_list=None, board_size: int | None = None,
                 n_frames: int | None = None, seed: int = 0, max_steps: int = 100000):
    """utils.jl:198-259: one SnakeGame() played to the end (epsilon-greedy, or
    the fixed `actions_list` of action indices). Returns (experiences,
    episode_reward, boards) where boards is the board history b_0..b_L;
    experiences["score"] is the game's score at the end (game.score)."""
    bs = board_size or model.board_size
    nf = n_frames or model.n_frames
    game = SnakeGame(bs, nf, n_envs=1, autoreset=True)
    rb = ReplayBuffer(max_steps + 1, board_size=bs, n_frames=nf, batch_size=1)
    act = DeviceArray(1, np.uint8)
    L, score = 0, 0
    while L < max_steps:
        if actions_list is not None:
            if L >= len(actions_list):
                break
            act.upload(np.array([actions_list[L]], np.uint8))
        else:
            call("snk_dqn_act", model.handle, game.handle, float(epsilon), int(seed), act.ptr)
        step_indices_dev(game, act.ptr, replay=rb)
        L += 1
        o = game.last("done", "score")
        score = int(o["score"][0])                           # game.score after this step (utils.jl:72)
        if o["done"][0]:
            break
    exp = stack_exp(rb, np.arange(L, dtype=np.int64))
    exp["score"] = score
    ep_reward = np.float32(0)
    for r in exp["rewards"]:
        ep_reward = np.float32(ep_reward + r)
    boards = [exp["states"][0][-1].astype(np.int8)] + [s[-1].astype(np.int8) for s in exp["next_states"]]
    return exp, float(ep_reward), np.stack(boards)
