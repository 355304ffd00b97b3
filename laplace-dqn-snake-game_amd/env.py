"""SnakeGame and the env methods, batched on the GPU.

Mirror of the reference's Julia API (structs.jl:33-99, utils.jl:7-149):
`SnakeGame(board_size, n_frames, discount, food_rng)` becomes a batch of
`n_envs` games that step in lockstep inside libsnakehip; `step!` is `step_`,
`reset!` is `reset_`, `virtual_step` reads the suicidal mask the fused step
kernel computed. Boards follow the reference's indexing: `game.board[e, i-1, j-1]`
is env e's Julia `board[i, j]` (-1 wall, 0 empty, 1 snake, 2 food).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import DeviceArray, call, ptr, vp

# utils.jl:8 order; CartesianIndex directions as (drow, dcol)
U, D, L, R = (-1, 0), (1, 0), (0, -1), (0, 1)
ALL_ACTIONS = (U, D, L, R)
DIR_CODE = {U: 0, D: 1, L: 2, R: 3}
NULL_ACTION = (0, 0)


def available_action_codes(prev_dir: int) -> list[int]:
    """utils.jl:7-10 — all four directions except the reverse of prev_dir."""
    return [a for a in range(4) if a != (prev_dir ^ 1)]


def food_list(board_size: int, seed: int = 42, n: int = 50) -> list[tuple[int, int]]:
    """structs.jl:70 food list as 1-based (row, col) pairs."""
    cells = np.zeros(n, np.int32)
    call("snk_food_list", board_size, seed, n, ptr(cells))
    return [(int(c) % board_size + 1, int(c) // board_size + 1) for c in cells]


class SnakeGame:
    """A batch of `n_envs` reference SnakeGame()s living in GPU memory.

    structs.jl:33 `SnakeGame(board_size=10, n_frames=2, discount=0.99,
    food_rng=Xoshiro(42))`. `autoreset=True` restarts a lost game on its next
    step (the batched trainer's mode); with False a lost game stays frozen
    until `reset_` (the reference's one-episode-per-SnakeGame() mode).
    """

    eating_reward = 1.0      # structs.jl:89
    suicide_penalty = -1.0   # structs.jl:90
    male_di_vivere = -0.01   # structs.jl:91

    def __init__(self, board_size: int = 10, n_frames: int = 2, discount: float = 0.99,
                 food_seed: int = 42, *, n_envs: int = 1, max_hist: int = 500, autoreset: bool = False):
        self.board_size = int(board_size)
        self.n_frames = int(n_frames)
        self.discount = float(discount)  # stored like the reference; unused (utils.jl:451 uses 0.97)
        self.food_seed = int(food_seed)
        self.n_envs = int(n_envs)
        self.max_hist = int(max_hist)
        self.autoreset = bool(autoreset)
        h = vp()
        call("snk_env_create", C.byref(h), self.n_envs, self.board_size, self.n_frames, self.food_seed,
             self.max_hist, int(self.autoreset))
        self._h = h
        self._act = DeviceArray(self.n_envs, np.uint8)
        outs = [vp() for _ in range(6)]
        call("snk_env_outputs", h, *[C.byref(o) for o in outs])
        self._out = dict(zip(("reward", "done", "mask", "dirs", "ep_reward", "score"),
                             (o.value for o in outs)))
        self.food_list = food_list(self.board_size, self.food_seed)

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.snk_env_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ state reads
    @property
    def board(self) -> np.ndarray:
        """[n_envs, bs, bs] int8, board[e, i-1, j-1] == Julia board[i, j]."""
        bs = self.board_size
        b = np.zeros((self.n_envs, bs * bs), np.int8)
        call("snk_env_get_boards", self._h, ptr(b))
        return np.swapaxes(b.reshape(self.n_envs, bs, bs), 1, 2)

    def board_cells(self) -> np.ndarray:
        """[n_envs, bs*bs] int8 in the reference's column-major memory order."""
        bs = self.board_size
        b = np.zeros((self.n_envs, bs * bs), np.int8)
        call("snk_env_get_boards", self._h, ptr(b))
        return b

    def _scalars(self):
        n = self.n_envs
        sc, ln, st, pd = (np.zeros(n, np.int32) for _ in range(4))
        lost = np.zeros(n, np.uint8)
        er = np.zeros(n, np.float32)
        call("snk_env_get_scalars", self._h, ptr(sc), ptr(ln), ptr(st), ptr(pd), ptr(lost), ptr(er))
        return dict(score=sc, len=ln, steps=st, prev_dir=pd, lost=lost.astype(bool), episode_reward=er)

    @property
    def score(self) -> np.ndarray:
        return self._scalars()["score"]

    @property
    def lost(self) -> np.ndarray:
        return self._scalars()["lost"]

    @property
    def prev_dir(self) -> list[tuple[int, int]]:
        return [ALL_ACTIONS[d] for d in self._scalars()["prev_dir"]]

    def snake(self, e: int = 0) -> list[tuple[int, int]]:
        """game.snake of env e as 1-based (row, col), head first."""
        bs = self.board_size
        cells = np.zeros(bs * bs, np.int32)
        n = C.c_int32(0)
        call("snk_env_get_snake", self._h, e, ptr(cells), C.byref(n))
        return [(int(c) % bs + 1, int(c) // bs + 1) for c in cells[:n.value]]

    # ------------------------------------------------------------ last step
    def last(self, *names: str) -> dict:
        """Host copies of the last step's outputs (reward, done, mask, dirs,
        ep_reward, score)."""
        n = self.n_envs
        types = dict(reward=np.float32, done=np.uint8, mask=np.uint8, dirs=np.uint8,
                     ep_reward=np.float32, score=np.uint8)
        names = names or tuple(types)
        return {k: _lib.view_numpy(self._out[k], n, types[k]) for k in names}

    def check_faults(self) -> int:
        c = C.c_int64(0)
        call("snk_env_check_faults", self._h, C.byref(c))
        return c.value

    @property
    def t(self) -> int:
        t = C.c_int64(0)
        call("snk_env_info", self._h, None, None, None, C.byref(t))
        return t.value


def available_actions(game: SnakeGame) -> list[list[tuple[int, int]]]:
    """utils.jl:7-10 per env: the three directions that are not a reversal."""
    return [[ALL_ACTIONS[a] for a in available_action_codes(pd)] for pd in game._scalars()["prev_dir"]]


def _upload_actions(game: SnakeGame, action):
    """Returns act_mode after writing the [n_envs] action bytes to the device."""
    if isinstance(action, tuple) and len(action) == 2 and all(isinstance(x, int) for x in action):
        action = [action] * game.n_envs
    a = action
    if isinstance(a, (list, tuple)) and len(a) and isinstance(a[0], tuple):
        codes = np.array([DIR_CODE[tuple(x)] for x in a], np.uint8)
        mode = _lib.SNK_ACT_DIRECTION
    else:
        codes = np.asarray(a, np.uint8).reshape(-1)
        if codes.size == 1 and game.n_envs > 1:
            codes = np.full(game.n_envs, codes[0], np.uint8)
        mode = _lib.SNK_ACT_INDEX
    assert codes.size == game.n_envs, "one action per env"
    game._act.upload(codes)
    return mode


def step_(game: SnakeGame, action, *, replay=None) -> None:
    """step! (utils.jl:100-109) for every env, fused with virtual_step.

    `action`: a direction tuple / list of direction tuples (the reference's
    CartesianIndex, absolute), or action indices 0..2 into
    available_actions. With `replay`, the transitions are store!d in the same
    kernel (requires autoreset)."""
    mode = _upload_actions(game, action)
    if replay is None:
        call("snk_env_step", game._h, game._act.ptr, mode)
    else:
        call("snk_env_step_store", game._h, game._act.ptr, mode, replay.handle)


def step_indices_dev(game: SnakeGame, act_dev_ptr, replay=None) -> None:
    """step! with action indices already on the device (no host traffic)."""
    if replay is None:
        call("snk_env_step", game._h, act_dev_ptr, _lib.SNK_ACT_INDEX)
    else:
        call("snk_env_step_store", game._h, act_dev_ptr, _lib.SNK_ACT_INDEX, replay.handle)


def virtual_step(game: SnakeGame):
    """utils.jl:112-132 — (available next actions, suicidal flags) per env for
    the state reached by the last step; a lost env gets [(0,0)]*3 and trues(3)."""
    o = game.last("mask", "dirs")
    out = []
    for m, d in zip(o["mask"], o["dirs"]):
        if (d >> 4) & 1:
            out.append(([NULL_ACTION] * 3, [True] * 3))
        else:
            av = [ALL_ACTIONS[a] for a in available_action_codes((d >> 2) & 3)]
            out.append((av, [bool((m >> k) & 1) for k in range(3)]))
    return out


def reset_(game: SnakeGame, mask=None) -> None:
    """reset!: SnakeGame() again for the envs where mask is true (all if None)."""
    m = None if mask is None else np.ascontiguousarray(np.asarray(mask, bool), np.uint8)
    call("snk_env_reset", game._h, ptr(m))


def assemble_state_(game: SnakeGame) -> np.ndarray:
    """assemble_state! (utils.jl:135-139): Float32 (bs, bs, n_frames, n_envs)
    Julia memory, i.e. [n_envs, n_frames, bs*bs] C-order, oldest frame first."""
    bs, nf = game.board_size, game.n_frames
    s = np.zeros((game.n_envs, nf, bs * bs), np.int8)
    call("snk_env_get_states", game._h, ptr(s))
    return s.astype(np.float32)


def synth_actions_dev(game: SnakeGame, seed: int, act: DeviceArray) -> None:
    """Counter-based synthetic action indices (bench / differential tests)."""
    call("snk_env_synth_actions", game._h, seed, act.ptr)
