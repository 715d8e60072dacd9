import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_cases(large=None, prefill=False):
    """Golden mul_mat cases; prefill=True selects the P_* cases (prefill-sized Y kept as its
    SHA-256 + sampled columns), which the other selections leave out."""
    cs = [c for c in load_manifest()["cases"] if c["name"].startswith("P_") == prefill]
    if large is None:
        return cs
    return [c for c in cs if bool(c["large"]) == large]


def golden_blob(name, dtype=np.uint8):
    return np.fromfile(os.path.join(GOLDEN, name), dtype=dtype)


@pytest.fixture(scope="session")
def manifest():
    return load_manifest()
