"""Kink-aware gradient parity (test infrastructure).

relu makes the loss gradient discontinuous where a pre-activation z is 0. An
fp32 device and the fp64 oracle agree on every decision except where z lies
within the device's rounding of 0, and a single such decision can move the
normwise gradient by ~1e-5 (the round-3 bench-graph run met one: a conv3
output at relative margin ~1e-7, b3 channel 60 off by 3.9e-6). When the
plain comparison misses, this helper proves the difference is such a kink and
nothing else: it re-runs the same batch through the device's training
forward/backward (bit-identical gradient required), reads the device's relu
decisions, and requires (1) the oracle gradient under THE DEVICE'S decisions
within the tolerance, and (2) every decision the device took differently to
sit at a kink: |z| <= 1e-5 * sum|terms| in the oracle's fp64 forward.
"""
import numpy as np

import oracle


def grad_parity(snk, m, bs, C, th, tt, batch, g_dev, tol=1e-5, restore=None, ref=None):
    """batch = (frames [B, C+1, nc] int8, act, rew, done, mask [B, 3]); ref =
    the oracle's dqn_loss_grad_kinks(...) on it if already computed.
    Returns (relative error vs the oracle's own decisions, relative error
    after kink accounting, number of kink decisions). Raises AssertionError
    when the difference is not explained by kinks."""
    f, ac, rw, dn, mk = batch
    B = f.shape[0]
    args = (bs, C, th, tt, f[:, :C], ac, rw, f[:, 1:], dn, mk)
    _, g_o, dec_o, mg_o = ref if ref is not None else oracle.dqn_loss_grad_kinks(*args)
    rg = float(np.linalg.norm(g_dev - g_o) / np.linalg.norm(g_o))
    if rg <= tol:
        return rg, rg, 0
    # replay the batch through the device's training path with the same parameters
    keep = restore() if restore else None
    rb = snk.ReplayBuffer(B, board_size=bs, n_frames=C, batch_size=B)
    snk.store_(rb, f, ac, rw, dn, mk, np.zeros(B, np.uint8))
    m.set_params(th)
    m.set_params(tt, snk.SNK_NET_TARGET)
    idx = snk.DeviceArray.from_host(np.arange(B, dtype=np.int64))
    m.loss_grad(rb, idx, B)
    assert np.array_equal(m.grad, g_dev), "the replayed batch must give the same device gradient"
    dec_d = m.train_relu_decisions(B)
    if keep is not None:
        keep()
    _, g_k, _, _ = oracle.dqn_loss_grad_kinks(*args, relu_in=dec_d)
    rk = float(np.linalg.norm(g_dev - g_k) / np.linalg.norm(g_k))
    diff = dec_d != dec_o
    n_kinks = int(diff.sum())
    worst_margin = float(np.abs(mg_o[diff]).max()) if n_kinks else 0.0
    assert rk <= tol, f"gradient off by {rk:.2e} even under the device's relu decisions ({n_kinks} differ)"
    assert n_kinks <= 16 and worst_margin <= 1e-5, (n_kinks, worst_margin)
    return rg, rk, n_kinks
