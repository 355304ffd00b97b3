"""Diagnostic: x6 split forward vs fp32 MFMA forward vs fp64 oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402
import snake_amd as snk  # noqa: E402

for bs, C, B, scale in [(12, 2, 300, 1.0), (12, 2, 300, 3.0), (10, 1, 257, 3.0)]:
    rng = np.random.default_rng(bs * 100 + B)
    m6 = snk.DQNModel(bs, 3, n_frames=C, seed=5)
    os.environ["SNK_CONV"] = "fp32"
    m32 = snk.DQNModel(bs, 3, n_frames=C, seed=5)
    del os.environ["SNK_CONV"]
    p = m6.get_params() * np.float32(scale)
    m6.set_params(p)
    m32.set_params(p)
    x = rng.integers(-1, 3, size=(B, C, bs * bs)).astype(np.float32)
    q6, q32 = m6.forward(x), m32.forward(x)
    qref = oracle.qnet_forward(bs, C, p, x)
    e6 = np.abs(q6 - qref) / np.maximum(1, np.abs(qref))
    e32 = np.abs(q32 - qref) / np.maximum(1, np.abs(qref))
    i6 = np.unravel_index(np.argmax(e6), e6.shape)
    print(bs, C, B, scale, "x6 max", e6.max(), "at", i6, q6[i6], qref[i6], "| fp32 max", e32.max(),
          "| mean", e6.mean(), e32.mean(), "| |q| max", np.abs(qref).max())
