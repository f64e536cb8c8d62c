"""Quick hardware probe: fp32 GEMM rate at DLRM MLP shapes, copy bandwidth, gather bandwidth."""
import time, torch, os
print("devices", torch.cuda.device_count(), torch.cuda.get_device_name(0), "cpus", len(os.sched_getaffinity(0)))
dev = "cuda"
def bench(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n
B = 65536
for (m, k, n) in [(B, 857, 512), (B, 512, 256), (B, 256, 1), (B, 13, 512), (B, 512, 256), (B, 256, 128), (857, B, 512), (512, B, 256)]:
    a = torch.randn(m, k, device=dev); b = torch.randn(k, n, device=dev)
    t = bench(lambda: a @ b)
    print(f"gemm {m}x{k}x{n}: {t*1e3:.1f} us  {2*m*k*n/t/1e9:.1f} TF/s")
x = torch.empty(2**28, device=dev); y = torch.empty_like(x)
t = bench(lambda: y.copy_(x))
print(f"copy 1GiB: {t:.3f} ms {2*x.numel()*4/t/1e6:.0f} GB/s")
tab = torch.randn(40_000_000, 128, device=dev)
idx = torch.randint(0, 40_000_000, (65536*26,), device=dev)
t = bench(lambda: tab.index_select(0, idx))
print(f"torch index_select 1.7M rows x512B: {t:.3f} ms {idx.numel()*512*2/t/1e6:.0f} GB/s")
