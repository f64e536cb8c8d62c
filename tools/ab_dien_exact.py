import sys
sys.path.insert(0, ".")
import torch
from recommender_amd import _lib as L
from recommender_amd.embedding import Embedding
import tests.test_dien_step_gpu as T

L.load()
orig = Embedding.take_grad
for skip in (1, 0):
    for mask in (True, False):
        L.RS_DIEN_SKIP_MASKED_ROWS = skip
        if mask:
            Embedding.take_grad = orig
        else:
            def tg(self, with_valid=False):
                r = orig(self, with_valid)
                return (r[0], r[1], None) if (r is not None and with_valid) else r
            Embedding.take_grad = tg
        try:
            T.test_dien_static_and_graph_step_equal_eager()
            print("skip", skip, "mask", mask, "OK", flush=True)
        except AssertionError as e:
            print("skip", skip, "mask", mask, "FAIL", str(e).splitlines()[:4], flush=True)
