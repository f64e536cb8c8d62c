import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: longer-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def lib():
    from recommender_amd import _lib as L

    return L.load()


@pytest.fixture
def rng():
    return np.random.default_rng(4)


def assert_close_rel(got, ref, rtol=1e-5, scale=None, msg=""):
    """|got - ref| <= rtol * (|ref| + scale): relative to the value, with a magnitude floor
    `scale` (e.g. the Cauchy-Schwarz bound of a dot product) so cancellations near zero are
    judged against the size of the terms that cancelled."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    if scale is None:
        scale = np.abs(ref).max() * 1e-3 if ref.size else 0.0
    err = np.abs(got - ref)
    bound = rtol * (np.abs(ref) + scale)
    bad = err > bound
    if bad.any():
        i = np.flatnonzero(bad.reshape(-1))[0]
        raise AssertionError(f"{msg} {bad.sum()} / {bad.size} elements off; first at {i}: "
                             f"got {got.reshape(-1)[i]!r} ref {ref.reshape(-1)[i]!r} "
                             f"(max err/bound {float((err / np.maximum(bound, 1e-300)).max()):.3g})")


from oracle.ctr import chain_grad_bounds  # noqa: E402,F401  (shared with oracle/check_dlrm.py)
