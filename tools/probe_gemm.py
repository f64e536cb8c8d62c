"""Probe fp32 weight-gradient GEMM options for the DLRM MLP shapes (K = batch = 65536)."""
import torch, time
dev = "cuda"
def bench(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3
B = 65536
shapes = [(857, 512), (512, 256), (256, 128), (13, 512), (256, 1), (128, 256)]
for lib in ["hipblas", "ck", "hipblaslt"]:
    if True:
        torch.backends.cuda.preferred_blas_library(lib)
    print("== backend", lib, torch.backends.cuda.preferred_blas_library())
    for (fi, fo) in shapes:
        x = torch.randn(B, fi, device=dev); dy = torch.randn(B, fo, device=dev)
        fl = 2 * B * fi * fo
        r = {}
        r["xT@dy"] = bench(lambda: x.t() @ dy)
        r["(dyT@x).T"] = bench(lambda: dy.t() @ x)
        for c in (16, 64):
            r[f"bmm split{c}"] = bench(lambda: torch.bmm(x.view(c, B // c, fi).transpose(1, 2), dy.view(c, B // c, fo)).sum(0))
        w = torch.randn(fi, fo, device=dev)
        r["fwd x@w"] = bench(lambda: x @ w)
        r["dx dy@wT"] = bench(lambda: dy @ w.t())
        print(f"[{fi}x{fo}] " + "  ".join(f"{k}={v:.0f}us({fl/v/1e6:.0f}TF)" for k, v in r.items()))
