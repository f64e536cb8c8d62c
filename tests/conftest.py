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


def assert_close_f64(got, ref64, ref32, msg="", rtol=1e-5, noise=4.0, floor=1e-7):
    """Per-element check of an fp32 result against a float64 evaluation of the same function:
    |got - ref64| <= rtol·|ref64| + noise·max_k|ref32_k - ref64| + floor·max|ref64|, where the
    ref32_k (one array or a list) are fp32 evaluations of the reference in different summation
    orders: their errors, element by element, stand for the rounding any fp32 evaluation order
    may show there; `floor` bounds the elements where those samples happen to be ~0."""
    def arr(x):
        x = x.detach().cpu().numpy() if hasattr(x, "detach") else x
        return np.asarray(x, np.float64)
    g, r = arr(got), arr(ref64)
    samples = ref32 if isinstance(ref32, (list, tuple)) else [ref32]
    spread = np.max([np.abs(arr(s) - r) for s in samples], axis=0)
    tol = rtol * np.abs(r) + noise * spread + floor * (np.abs(r).max() if r.size else 0.0)
    err = np.abs(g - r)
    bad = ~(err <= tol)
    if bad.any():
        i = int(np.flatnonzero(bad.reshape(-1))[0])
        raise AssertionError(f"{msg}: {int(bad.sum())} / {bad.size} elements off; first at {i}: "
                             f"got {g.reshape(-1)[i]!r} ref {r.reshape(-1)[i]!r} "
                             f"(max err/tol {float((err / np.maximum(tol, 1e-300)).max()):.3g})")


def run_ranks(target, world, args=(), timeout=300):
    """Spawn `world` processes target(rank, world, *args, q) and collect one (rank, status) each
    from the queue; fails as soon as a rank dies without reporting (no silent wait for the
    whole timeout) and prints a heartbeat while waiting. Returns {rank: status}."""
    import queue as _queue
    import time as _time

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world, *args, q)) for r in range(world)]
    for p in ps:
        p.start()
    res, t0, beat = {}, _time.time(), _time.time()
    try:
        while len(res) < world:
            try:
                r, v = q.get(timeout=5)
                res[r] = v
                continue
            except _queue.Empty:
                pass
            dead = [i for i, p in enumerate(ps) if p.exitcode not in (None, 0) and i not in res]
            if dead:
                raise AssertionError(f"rank(s) {dead} died (exit {[ps[i].exitcode for i in dead]}) "
                                     f"before reporting; got {res}")
            if _time.time() - t0 > timeout:
                raise AssertionError(f"ranks did not report within {timeout} s; got {res}")
            if _time.time() - beat > 30:
                print(f"[run_ranks] waiting: {len(res)}/{world} reported after "
                      f"{_time.time() - t0:.0f} s", flush=True)
                beat = _time.time()
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    return res
