"""Synthetic Criteo TSV text for the ingestion tests (not a test module)."""
import numpy as np


def make_tsv(rng, n_lines=400, vocab=60, crlf_every=7, trailing_newline=False):
    toks = [f"{rng.integers(0, 2**32):08x}" for _ in range(vocab)]
    lines = []
    for k in range(n_lines):
        label = str(int(rng.random() < 0.25))
        ints = []
        for _ in range(13):
            r = rng.random()
            ints.append("" if r < 0.1 else str(-int(rng.integers(1, 5))) if r < 0.15
                        else str(int(rng.geometric(0.01))))
        cats = []
        for c in range(26):
            r = rng.random()
            cats.append("" if r < 0.08 else toks[min(int(rng.zipf(1.3)) - 1, vocab - 1)])
        if k % 11 == 0:
            cats[25] = cats[0] or toks[0]  # same token in C1 and C26 (distinct vocab keys)
        lines.append("\t".join([label] + ints + cats))
    text = ""
    for k, ln in enumerate(lines):
        last = k == len(lines) - 1
        text += ln + ("" if last and not trailing_newline else ("\r\n" if k % crlf_every == 3 else "\n"))
    return text
