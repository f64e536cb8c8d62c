"""Generate the golden fixtures in tests/golden/ from the NumPy oracle (oracle/*.py).

The reference (TensorFlow 2.2 / DGL) is not importable here, and the reference ships no
fixtures, so these vectors pin the oracle's restatement — they are checked by
the CPU tests against the oracle and by the GPU tests against the HIP kernels. Regenerate with
`python tests/golden/make_golden.py` (deterministic, seed 4)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import embedding as OE  # noqa: E402
from oracle import interaction as OI  # noqa: E402
from oracle import pinsage as OP  # noqa: E402


def zipf_ids(rng, n, card):
    return np.minimum(rng.zipf(1.05, size=n) - 1, card - 1)


def main():
    rng = np.random.default_rng(4)
    # a-1/a-2: slab lookup, sort, tiled segmented sum, SGD / lazy / keras Adam on touched rows
    card = np.array([7, 1, 300, 1000, 50])
    so = np.concatenate([[0], np.cumsum(card)]).astype(np.int64)
    V, D, B = int(so[-1]), 16, 700
    ids = np.stack([zipf_ids(rng, B, c) for c in card], 1).astype(np.int64)
    ids[5, 1] = 3  # OOB for the 1-row slot
    table = rng.standard_normal((V, D)).astype(np.float32)
    grad = rng.standard_normal((ids.size, D)).astype(np.float32)
    emb = OE.embedding_lookup(table, ids, so, raise_oob=False)
    sr, sp, nu = OE.sort_ids(ids, V, so)
    ur, ug = OE.segment_sum_tiled(sr, sp, grad, V)
    c = OE.keras_adam_coefficients(1)
    m = np.zeros_like(table)
    v = np.zeros_like(table)
    sgd = OE.apply_sgd(table, ur, ug, np.float32(0.05))
    lz = OE.apply_lazy_adam(table, m, v, ur, ug, c)
    ka = OE.apply_keras_adam(table, m, v, ur, ug, c)
    np.savez_compressed(os.path.join(HERE, "embedding.npz"), slot_offsets=so, ids=ids, table=table,
                        grad=grad, emb=emb, sorted_rows=sr, sorted_pos=sp, n_unique=nu,
                        uniq_rows=ur, uniq_grad=ug, sgd=sgd, lazy_w=lz[0], lazy_m=lz[1],
                        lazy_v=lz[2], keras_w=ka[0], keras_m=ka[1], keras_v=ka[2])
    # a-4/a-5: DotInteraction (4 modes), DLRM fused, FM
    x = rng.standard_normal((9, 27, 32)).astype(np.float32)
    out = {"x": x}
    for si in (0, 1):
        for sg in (0, 1):
            z = OI.dot_interaction(x, bool(si), bool(sg))
            g = rng.standard_normal(z.shape).astype(np.float32)
            out[f"z_{si}{sg}"] = z
            out[f"g_{si}{sg}"] = g
            out[f"gx_{si}{sg}"] = OI.dot_interaction_bwd(x, g, bool(si), bool(sg))
    e = rng.standard_normal((9, 26, 16)).astype(np.float32)
    ge = rng.standard_normal(9).astype(np.float32)
    out.update(fm_e=e, fm_out=OI.fm(e), fm_g=ge, fm_ge=OI.fm_bwd(e, ge))
    np.savez_compressed(os.path.join(HERE, "interaction.npz"), **out)
    pinsage_fixture()
    print("wrote", os.listdir(HERE))


def pinsage_fixture():
    """a-14..a-16: a 40-user / 70-item graph with dead ends; one step of pairs + 2-layer
    blocks (walk params (2, 4, 0, 3) of pinsage/train/train.py:69) with leak-edge removal."""
    rng = np.random.default_rng(4)
    u = rng.integers(0, 36, 300)
    i = rng.integers(0, 64, 300)
    key = np.unique(u * 70 + i)
    users, items = key // 70, key % 70
    g = OP.BipartiteGraph.from_edges(users, items, 40, 70)
    seed, step = 4, 2
    h, p, n = OP.item_pairs(g, 0, 48, seed, step)
    seeds, pe, ne, blocks = OP.sample_from_item_pairs(g, h, p, n, 2, 4, 2, 0.0, 3, seed, step)
    out = dict(users=users, items=items, heads=h, pos=p, neg=n, seeds=seeds, pos_src=pe[0],
               pos_dst=pe[1], neg_dst=ne[1])
    for li, b in enumerate(blocks):
        for f in ("src_nodes", "indptr", "edge_src", "edge_dst", "edge_w", "t_indptr", "t_edge"):
            out[f"b{li}_{f}"] = getattr(b, f)
    np.savez_compressed(os.path.join(HERE, "pinsage.npz"), **out)


if __name__ == "__main__":
    main()
