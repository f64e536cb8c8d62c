"""Synthetic Ali-CCP and Amazon (DIEN) text for the ingestion tests (not a test module)."""
import numpy as np

from oracle.textpipe import ALICCP_COLUMNS

_EXTRA_FIELDS = ["150_14", "109_14", "110_14", "999"]


def _feat(field, value, rng):
    return f"{field}\x02{value}\x03{rng.random():.4f}"


def _kv(rng, fields, p_present, n_vals, dup_p=0.1):
    feats = []
    for f in fields:
        if rng.random() < p_present:
            feats.append(_feat(f, 1000 + min(int(rng.zipf(1.4)), n_vals), rng))
            if rng.random() < dup_p:  # a repeated field: the later value wins (dict(zip))
                feats.append(_feat(f, 1000 + min(int(rng.zipf(1.4)), n_vals), rng))
    order = rng.permutation(len(feats))
    return "\x01".join(feats[i] for i in order)


def make_aliccp(rng, n_skel=600, n_common=40, n_vals=30, crlf_every=9):
    """(skeleton_text, common_text). Columns split between skeleton and common features as in
    the dataset (user-side fields in the common file), with overlaps so the common value must
    override; some skeleton lines are (click 0, purchase 1) and get dropped."""
    cols = ALICCP_COLUMNS + _EXTRA_FIELDS
    user_cols = cols[:9] + ["150_14", "109_14", "301"]
    common_lines = []
    for k in range(n_common):
        common_lines.append(f"c{k:05x},{len(user_cols)},{_kv(rng, user_cols, 0.8, n_vals)}")
    common_lines.append(f"c{0:05x},1,{_feat('101', 4242, rng)}")  # a duplicate id: later wins
    skel_lines = []
    for k in range(n_skel):
        r = rng.random()
        click, buy = (0, 1) if r < 0.05 else (1, int(rng.random() < 0.3)) if r < 0.3 else (0, 0)
        kv = _kv(rng, cols[9:] + ["101", "301"], 0.7, n_vals)
        if k % 37 == 5:
            kv += "\x01" + "216"  # a trailing key with no value: zip drops it
        if k % 53 == 7:
            kv = ""
        skel_lines.append(f"s{k},{click},{buy},c{int(rng.integers(0, n_common)):05x},5,{kv}")

    def join(lines):
        out = ""
        for k, ln in enumerate(lines):
            out += ln + ("\r\n" if k % crlf_every == 4 else "\n")
        return out

    return join(skel_lines), join(common_lines)


def make_amazon(rng, n_lines=500, n_items=80, n_cats=12, max_hist=140, unseen_items=0,
                trailing_newline=True):
    """DIEN lines; the item → cat map changes over time (the last pair wins); `unseen_items`
    adds items outside the training vocabulary (→ unk) keeping cats known."""
    cat_of = rng.integers(0, n_cats, n_items + unseen_items)
    lines = []
    for k in range(n_lines):
        if k == n_lines // 2:
            cat_of[:5] = (cat_of[:5] + 1) % n_cats
        L = int(min(1 + rng.geometric(0.05), max_hist)) if k % 17 else 1
        hi = [min(int(rng.zipf(1.3)) - 1, n_items + unseen_items - 1) for _ in range(L)]
        tgt = int(rng.integers(0, n_items + unseen_items))
        his_items = "\x02".join(f"I{x}" for x in hi)
        his_cats = "\x02".join(f"C{cat_of[x]}" for x in hi)
        lines.append("\t".join([str(int(rng.random() < 0.5)), f"U{k % 50}", f"I{tgt}",
                                f"C{cat_of[tgt]}", his_items, his_cats]))
    text = "\n".join(lines)
    return text + ("\n" if trailing_newline else "")
