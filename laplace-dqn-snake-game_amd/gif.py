"""Best-game GIF export (utils.jl:628-675, 680-701): the board history of one
episode rendered in the reference's own GIF format.

The reference animates `game.board_history` with Plots.jl (`plot_board`,
utils.jl:655-675: white background, walls black, snake green, food red) into
a 600 x 400 canvas where each board cell is a 36 px square and a 10 x 10
board's top-left corner sits at pixel (x 131, y 12), with a light-grey
frame line above it; `gif(anim, path, fps=1)`. This module writes that
format from the device's boards (the episode itself runs in libsnakehip), so
tests/golden/make_fixtures.py's decoder reads our GIFs and the reference's
alike. Host-side rendering only: it is analysis output, not the hot path.
"""
from __future__ import annotations

import os

import numpy as np

W, H = 600, 400
CELL10, X0_10, Y0_10 = 36, 131, 12            # the reference's 10 x 10 geometry
COLOURS = {-1: (0, 0, 0), 0: (255, 255, 255), 1: (0, 255, 0), 2: (255, 0, 0)}
FRAME_GREY = (207, 207, 207)


def geometry(bs: int) -> tuple[int, int, int]:
    """(cell px, x0, y0): the 10 x 10 layout exactly; other boards keep the
    360 px square, centred on the same point."""
    if bs == 10:
        return CELL10, X0_10, Y0_10
    cell = 360 // bs
    side = cell * bs
    return cell, X0_10 + (360 - side) // 2, Y0_10 + (360 - side) // 2


def render_board(board: np.ndarray) -> np.ndarray:
    """plot_board (utils.jl:655-675): board[i, j] (row-major, 1 = top row) ->
    RGB uint8 [400, 600, 3]."""
    board = np.asarray(board)
    bs = board.shape[0]
    cell, x0, y0 = geometry(bs)
    img = np.full((H, W, 3), 255, np.uint8)
    img[y0 - 1, x0:x0 + bs * cell] = FRAME_GREY
    lut = np.zeros((4, 3), np.uint8)
    for v, c in COLOURS.items():
        lut[v + 1] = c
    px = lut[board.astype(np.int64) + 1]                       # [bs, bs, 3]
    img[y0:y0 + bs * cell, x0:x0 + bs * cell] = np.repeat(np.repeat(px, cell, 0), cell, 1)
    return img


def cells_to_board(cells: np.ndarray, bs: int) -> np.ndarray:
    """Column-major cells (cell = (i-1) + (j-1)*bs) -> row-major board[i, j]."""
    return np.asarray(cells).reshape(bs, bs).T


def board_history(boards_cells: np.ndarray, n_frames: int) -> np.ndarray:
    """game.board_history of an episode with boards b_0..b_L: n_frames copies
    of b_0 (structs.jl:53), one board per step (utils.jl:106), then n_frames-1
    copies of the last (utils.jl:229)."""
    b = np.asarray(boards_cells)
    return np.concatenate([np.repeat(b[:1], n_frames, 0), b[1:], np.repeat(b[-1:], n_frames - 1, 0)])


_PALETTE = [(255, 255, 255), (0, 0, 0), (0, 255, 0), (255, 0, 0), FRAME_GREY, (0, 0, 0), (0, 0, 0), (0, 0, 0)]


def _frame_block(img_rgb: np.ndarray) -> tuple[bytes, bytes]:
    """One frame as a GIF image block (descriptor + LZW data) under the fixed
    8-colour global palette; also returns the global colour table bytes."""
    import io

    from PIL import Image
    idx = np.zeros(img_rgb.shape[:2], np.uint8)
    for k, c in enumerate(_PALETTE[:5]):
        idx[(img_rgb == np.array(c, np.uint8)).all(-1)] = k
    im = Image.fromarray(idx, mode="P")
    im.putpalette([v for c in _PALETTE for v in c])
    buf = io.BytesIO()
    im.save(buf, format="GIF", optimize=False)
    b = buf.getvalue()
    flags = b[10]
    gct_len = 3 * (2 << (flags & 7)) if flags & 0x80 else 0
    gct = b[13:13 + gct_len]
    p = 13 + gct_len
    while b[p] == 0x21:                      # skip extensions: label, sub-blocks, terminator
        p += 2
        while b[p]:
            p += b[p] + 1
        p += 1
    assert b[p] == 0x2C, "GIF image descriptor expected"
    q = p + 10
    if b[p + 9] & 0x80:
        q += 3 * (2 << (b[p + 9] & 7))
    q += 1                                   # LZW minimum code size
    while b[q]:
        q += b[q] + 1
    return b[p:q + 1], gct


def save_gif(history_cells: np.ndarray, bs: int, path: str, fps: int = 1) -> str:
    """`gif(anim, path, fps=fps)` of a board history (column-major cells): one
    GIF frame per board, repeats included (the reference's board_history
    starts with n_frames copies of b_0), delay 1/fps s, looping."""
    import struct
    blocks, gct = [], b""
    for c in history_cells:
        blk, gct = _frame_block(render_board(cells_to_board(c, bs)))
        blocks.append(blk)
    delay = int(round(100 / fps))
    out = bytearray(b"GIF89a")
    out += struct.pack("<HHBBB", W, H, 0x80 | 0x70 | ((len(gct) // 3).bit_length() - 2), 0, 0)
    out += gct
    out += b"\x21\xff\x0bNETSCAPE2.0\x03\x01\x00\x00\x00"   # loop forever
    for blk in blocks:
        out += b"\x21\xf9\x04\x00" + struct.pack("<H", delay) + b"\x00\x00"
        out += blk
    out += b"\x3b"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(bytes(out))
    return path


def play_best_game(tr_or_model, name: str | None = None, path: str = "./trainer_gifs/", fps: int = 1):
    """utils.jl:628-652: one greedy episode (epsilon 0) of the trainer's (or
    the given) model on the device, animated; `name` given: saved as
    path/name.gif. Returns (score, episode_reward, board_history cells)."""
    from .trainer import play_episode
    model = getattr(tr_or_model, "model", tr_or_model)
    exp, ep_reward, boards = play_episode(model, 0.0)
    hist = board_history(boards, model.n_frames)
    score = exp["score"]   # the device's game.score: an eat on a losing step still counts (utils.jl:72, :90)
    if name is not None:
        save_gif(hist, model.board_size, os.path.join(path, name + ".gif"), fps=fps)
    return score, ep_reward, hist


def play_episode_with_animation(actions_list, *, model, epsilon: float = 0.0, gif_name: str | None = None,
                                fps: int = 1, path: str = "./gifs/"):
    """utils.jl:678-701: play_episode with a fixed list of action indices,
    animated; returns (experiences, episode_reward, board_history cells)."""
    from .trainer import play_episode
    exp, ep_reward, boards = play_episode(model, epsilon, actions_list=list(actions_list))
    hist = board_history(boards, model.n_frames)
    if gif_name is not None:
        save_gif(hist, model.board_size, os.path.join(path, gif_name + ".gif"), fps=fps)
    return exp, ep_reward, hist
