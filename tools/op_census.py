"""Which torch ops a model's graph-captured step records besides the engine's kernels: runs one
eager static_step of the cfg3 DIEN (or one step of --model esmm / mmoe at cfg4 size, or a PinSage static step with its sampling) under torch.profiler (CPU
activity only: the aten calls, with input shapes) and prints the count and shapes of the
memory-moving glue (add, copy_, cat, stack, fill_, zero_, clone, contiguous, mul, sum). Every
such call is one kernel / memcpy node in the replayed graph. GPU box: python tools/op_census.py"""
import argparse
import collections
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommender_amd import _lib as L  # noqa: E402

GLUE = ("aten::add", "aten::add_", "aten::copy_", "aten::cat", "aten::stack", "aten::fill_",
        "aten::zero_", "aten::clone", "aten::mul", "aten::mul_", "aten::sum", "aten::sub",
        "aten::div", "aten::where", "aten::neg", "aten::_foreach_copy_", "aten::mean",
        "aten::clamp", "aten::index_select", "aten::to", "aten::ones_like", "aten::zeros_like")


def dien_step():
    from recommender_amd.dien import DIEN
    from recommender_amd.dien.train import DIENStep, synthetic_batch
    from recommender_amd.gemm_tuning import use_tuned_gemms

    use_tuned_gemms()
    rng = np.random.default_rng(4)
    m = DIEN(36, 36, item_vocab_size=63001, item_embedding_size=18, cat_vocab_size=801,
             cat_embedding_size=18, mlp_units=[200, 80, 1], device="cuda")
    step = DIENStep(m)
    f, lab = synthetic_batch(rng, 4096, 100, 63001, 801)
    feats = {k: torch.from_numpy(v).cuda() for k, v in f.items()}
    label = torch.from_numpy(lab).cuda()
    return lambda: step.static_step(feats, label)


def multitask_step(name):
    from recommender_amd.esmm import FEAT_VOCAB
    from recommender_amd.esmm.train import MultiTaskStep, build
    from recommender_amd.gemm_tuning import use_tuned_gemms
    from recommender_amd.synthetic import aliccp_batch, scaled_vocab

    use_tuned_gemms()
    rng = np.random.default_rng(4)
    vocab = scaled_vocab(FEAT_VOCAB, 40_000_000)
    m = build(name.upper(), vocab, 18, "cuda")
    step = MultiTaskStep(m, "lazy_adam")
    f, lab = aliccp_batch(rng, 65536, vocab)
    feats = {k: torch.from_numpy(v).cuda() for k, v in f.items()}
    label = torch.from_numpy(lab).cuda()
    return lambda: step(feats, label)


def pinsage_step():
    from recommender_amd.pinsage import PinSageModel, PinSageSampler
    from recommender_amd.pinsage.train import ML20M, PinSageStep, build_graph

    g = build_graph(ML20M, 4)
    m = PinSageModel(g, g.itype, 2, 8, 32, 16)
    train = PinSageStep(m)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    ctr = {"it": 0}

    def fn():
        ctr["it"] += 1
        return train.static_step(*smp.sample_static(*smp.sample_pairs_static(4096, 4, ctr["it"])))
    return fn


def deepfm_step():
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch

    rng = np.random.default_rng(4)
    m = build_model("DeepFM", 16, 1_000_000, 26, 13, "cuda")
    step = TrainStep(m, "keras_adam", fused=False)
    cat, dn, lb = criteo_batch(rng, 1024, [1_000_000] * 26)
    batch = (torch.from_numpy(cat).cuda(), torch.from_numpy(dn).cuda(), torch.from_numpy(lb).cuda())
    return lambda: step.static_step(batch)


def eges_step():
    from recommender_amd.eges.train import EGESStep, build, synthetic_batch

    rng = np.random.default_rng(4)
    m = build("EGES", 63001, 801, 3000, 160)
    step = EGESStep(m)
    *inp, lab = synthetic_batch(rng, 1024, 63001, 801, 3000)
    inp = tuple(torch.from_numpy(a).cuda() for a in inp)
    lab = torch.from_numpy(lab).cuda()
    return lambda: step.static_step(inp, lab)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="dien", choices=["dien", "esmm", "mmoe", "pinsage", "deepfm", "eges"])
    args = ap.parse_args()
    L.load()
    fn = {"dien": dien_step, "pinsage": pinsage_step, "deepfm": deepfm_step,
          "eges": eges_step}.get(
        args.model, lambda: multitask_step(args.model))()
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
        fn()
        torch.cuda.synchronize()
    cnt = collections.Counter()
    shapes = collections.defaultdict(collections.Counter)
    # only top-level glue: an op whose parent is itself glue (e.g. copy_ inside cat) is skipped
    for ev in prof.events():
        if ev.name not in GLUE:
            continue
        parent = ev.cpu_parent
        if parent is not None and parent.name in GLUE:
            continue
        cnt[ev.name] += 1
        shapes[ev.name][str(ev.input_shapes)[:150]] += 1
    total = 0
    for name, n in cnt.most_common():
        total += n
        print(f"{n:4d}  {name}")
        for s, k in shapes[name].most_common(12):
            print(f"        {k:3d} x {s}")
    print(f"{total} glue calls in one step")


if __name__ == "__main__":
    main()
