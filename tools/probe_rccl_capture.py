"""Probe: which torch.distributed collectives on RCCL survive HIP graph capture on this image
(world 1 nccl group, the collective issued on a side stream forked from the capture stream, as
the sharded exchange does). One collective kind per process: python tools/probe_rccl_capture.py
<all_reduce|all_to_all|all_gather|a2a_main|copy_side|copy_main|record_side|alloc_side>"""
import os
import sys
from datetime import timedelta

import torch
import torch.distributed as dist

kind = sys.argv[1]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0),
                        timeout=timedelta(seconds=60))
x = torch.arange(4096, dtype=torch.float32, device="cuda")
y = torch.empty_like(x)
side = torch.cuda.Stream()


def op():
    if kind == "all_reduce":
        dist.all_reduce(x)
    elif kind == "all_gather":
        dist.all_gather_into_tensor(y, x)
    elif kind in ("all_to_all", "a2a_main"):
        dist.all_to_all_single(y, x)
    elif kind in ("copy_side", "copy_main"):
        y.copy_(x)  # a device-to-device copy (hipMemcpyAsync)
    elif kind == "record_side":  # record_stream of tensors allocated before the capture
        y.copy_(x)
        x.record_stream(torch.cuda.current_stream())
        y.record_stream(torch.cuda.current_stream())
    elif kind == "alloc_side":  # a tensor allocated on the side stream inside the capture, freed
        t = torch.empty_like(x)
        t.copy_(x)
        y.copy_(t)
        t.record_stream(torch.cuda.current_stream())
        del t


def body():
    if kind in ("a2a_main", "copy_main"):
        op()
        return
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        op()
    cur.wait_stream(side)


body()  # eager first (communicator init)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
print(kind, "captured", flush=True)
g.replay()
torch.cuda.synchronize()
print(kind, "replayed ok", flush=True)
dist.destroy_process_group()
