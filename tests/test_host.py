"""CPU tests of host logic and the C-ABI boundary (library loads, exports every symbol
include/recsys_hip.h declares, rejects bad arguments without touching a GPU)."""
import ctypes as C

import numpy as np
import pytest

from recommender_amd import _lib as L


def test_library_exports_header_symbols(lib):
    syms = L.header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.rs_version() >= 1


def test_every_header_symbol_has_a_python_signature():
    assert set(L.header_symbols()) <= set(L._SIGS)


def test_build_id_matches_sources_and_stale_library_is_refused(lib):
    from recommender_amd.build import source_hash

    assert lib.rs_build_id().decode() == source_hash()

    class Stale:
        @staticmethod
        def rs_build_id():
            return b"0000000000000000"

    with pytest.raises(L.RecsysError, match="other sources"):
        L.check_build_id(Stale(), "stale.so")


def test_argument_validation_without_gpu(lib):
    # null table with n_ids > 0 → RS_E_INVALID and a message, no device access
    st = lib.rs_embedding_fwd(None, 10, 4, None, 1, 5, None, 1, None, None, None)
    assert st == -1
    assert b"null" in lib.rs_last_error()
    assert lib.rs_embedding_fwd(None, 10, 0, None, 1, 5, None, 1, None, None, None) == -1
    assert lib.rs_dot_interaction_fwd(None, 4, 3, 8, 0, 1, None, 2, None) == -1  # stride < F*F
    with pytest.raises(L.RecsysError):
        L.check(-1, "rs_x")


def test_workspace_queries(lib):
    assert lib.rs_sort_ids_workspace_size(1 << 20) > 8 << 20
    assert lib.rs_apply_workspace_size(1 << 20, 128) >= (1 << 20) // 32 * 2 * 128 * 4


def test_no_cpu_fallback():
    import torch

    from recommender_amd.functional import dot_interaction

    with pytest.raises(L.RecsysError):
        dot_interaction(torch.zeros(2, 3, 4), False, True)


def test_dlrm_scheduler_matches_reference_formula():
    from recommender_amd.optim import DLRMScheduler

    s = DLRMScheduler(0.01, 20, 10000, 0.0001)
    assert s(0) == 0.0
    assert abs(s(10) - 0.005) < 1e-9
    assert abs(s(20) - 0.01) < 1e-9
    mid = s(20 + 5000)
    assert abs(mid - 0.01 * ((1 - 1e-4) * 0.5 * (1 + np.cos(np.pi * 0.5)) + 1e-4)) < 1e-7
    assert abs(s(10 ** 6) - 0.01 * 1e-4) < 1e-9


def test_keras_adam_coefficients_host():
    from oracle.embedding import keras_adam_coefficients as ref
    from recommender_amd.optim import keras_adam_coefficients

    for t in (1, 7, 100):
        assert np.float32(keras_adam_coefficients(t).lr) == ref(t)["lr"]


def test_criteo_cardinalities_and_ids():
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    c = criteo_cardinalities()
    assert len(c) == 26 and sum(c) == 40_000_000
    rng = np.random.default_rng(4)
    cat, dn, lb = criteo_batch(rng, 4096, c)
    assert cat.shape == (4096, 26) and (cat >= 0).all() and (cat < np.array(c)).all()
    assert dn.shape == (4096, 13) and abs(lb.mean() - 0.256) < 0.03


def test_graph_keras_adam_flat_layout_cpu():
    """GraphKerasAdam's flat buffers (host logic only, no kernel call): every parameter becomes a
    16-byte-aligned view of `flat` with its values kept, and grad_view(i) is the same slice of
    `grad_flat`, so a densified gradient written there lands where rs_keras_adam_flat reads it
    and the padding between parameters stays 0."""
    import torch

    from recommender_amd.optim import GraphKerasAdam

    ps = [torch.nn.Parameter(torch.arange(n, dtype=torch.float32).reshape(shape))
          for n, shape in ((6, (2, 3)), (5, (5,)), (8, (4, 2)))]
    want = [p.detach().clone() for p in ps]
    opt = GraphKerasAdam(ps, lr=1e-3, window=4)
    for i, (p, w) in enumerate(zip(ps, want)):
        assert torch.equal(p.detach(), w)
        o, n, pad = opt._segs[i]
        assert o % 4 == 0 and (n + pad) % 4 == 0
        assert p.data_ptr() == opt.flat[o:].data_ptr()
        gv = opt.grad_view(i)
        assert gv.shape == p.shape and gv.data_ptr() == opt.grad_flat[o:].data_ptr()
        gv.fill_(float(i + 1))
    pad_mask = torch.ones_like(opt.grad_flat, dtype=torch.bool)
    for i, (o, n, _) in enumerate(opt._segs):
        assert torch.all(opt.grad_flat[o:o + n] == float(i + 1))
        pad_mask[o:o + n] = False
    assert torch.all(opt.grad_flat[pad_mask] == 0)


def test_bench_pmc_filter_keeps_every_family_main_kernel():
    """bench.py's PMC passes filter kernels by PMC_KERNEL_REGEX and count each family's calls by
    its main kernel: a main kernel the filter drops leaves the family at 0 calls and the line's
    traffic null (a round-5 regression: the slot-segmented sort's kernels were filtered out)."""
    import re

    import bench

    for entry, _, main in bench.PMC_SYMBOLS:
        for alt in main.split("|"):
            name = "void rs::" + re.sub(r"\\d\+", "9", alt).replace("\\", "") + "(...)"
            assert re.search(bench.PMC_KERNEL_REGEX, name), (entry, alt)
