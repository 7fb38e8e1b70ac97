"""Shared test setup.

Markers: ``gpu`` = needs an MI355X (run on the GPU box with ``-m gpu``);
everything else runs on the CPU-only build container.
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP path)")


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_case(name):
    """A fixture's arrays. Large fixtures omit b, which every case draws as
    default_rng(1).standard_normal(N) (tests/golden/make_golden.py)."""
    import numpy as np
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    if "b" not in g:
        g["b"] = np.random.default_rng(1).standard_normal(g["x"].size)
    return g


def golden_matrix(spec):
    from oracle import matrices
    if spec[0] == "poisson":
        return matrices.poisson(spec[1], spec[2])
    return matrices.banded(*spec[1:])


@pytest.fixture(scope="session")
def manifest():
    return golden_manifest()
