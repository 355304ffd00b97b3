import os
import sys

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    import json
    out = {}
    with open(os.path.join(GOLDEN, "bson_vanilla.json")) as f:
        out["bson"] = json.load(f)
    out["double3"] = dict(np.load(os.path.join(GOLDEN, "gif_double3.npz")))
    out["vanilla1"] = dict(np.load(os.path.join(GOLDEN, "gif_vanilla1.npz")))
    out["vanilla_params"] = np.load(os.path.join(GOLDEN, "vanilla_qnet_params.npy"))
    out["vanilla_q"] = np.load(os.path.join(GOLDEN, "vanilla_q_fp64.npy"))
    return out


@pytest.fixture(scope="session")
def snk():
    """The product package, with a HIP device required."""
    import snake_amd
    snake_amd.load()
    if snake_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return snake_amd
