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


def chain_grad_bounds(x, layers, G):
    """Float64 magnitude bounds of an MLP chain's parameter gradients for BOTH evaluation
    orders (layer by layer, or factored from the last layer's G): h_{l-1} = x·R + c, so
    |h_{l-1}ᵀ·g_l| <= (|R|ᵀ·|x|ᵀ·|G| + |c|⊗Σ|G|)·|Q_l|ᵀ with Q_l = K_{l+1}···K_L.
    layers = [(kernel [in, out], bias [out])] as the input sees them (float64); G [B, n_L].
    Returns ([(kernel bound, bias bound)] per layer, dx bound [B, in])."""
    aG = np.abs(np.asarray(G, np.float64))
    base = np.abs(np.asarray(x, np.float64)).T @ aG
    Mb, absR, absc = [], None, None
    for i, (k, b) in enumerate(layers):
        Mb.append(base if i == 0 else absR.T @ base + np.outer(absc, aG.sum(0)))
        absR = np.abs(k) if absR is None else absR @ np.abs(k)
        absc = np.abs(b) if absc is None else np.abs(k).T @ absc + np.abs(b)
    out = [None] * len(layers)
    absQ = None
    for i in range(len(layers) - 1, -1, -1):
        kb, bb = Mb[i], aG.sum(0)
        if absQ is not None:
            kb, bb = kb @ absQ.T, bb @ absQ.T
        out[i] = (kb, bb)
        absQ = np.abs(layers[i][0]) if absQ is None else np.abs(layers[i][0]) @ absQ
    return out, aG @ absQ.T
