"""Join tools/pinsage_prof.sh's kernel stats and PMC passes: per PinSage kernel, the average
duration in the graph step, the HBM bytes per launch from FETCH_SIZE (x2, the gfx950 16-B read
correction) + WRITE_SIZE, and the achieved GB/s against the 8 TB/s peak."""
import csv
import glob
import re
from collections import defaultdict

KERNELS = ["neighbors_kernel", "agg_fwd_kernel", "agg_bwd_kernel", "block_emit_kernel",
           "first_mark_kernel", "first_emit_kernel", "walk_kernel", "pairs_gen_kernel",
           "pair_margin_fwd_kernel", "pair_margin_terms_kernel", "multihot_mean_fwd",
           "multihot_mean_bwd"]


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


stats = {}
for f in glob.glob("gpurun_out/pin_kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Name"])
        if k:
            n, tot = stats.get(k, (0, 0.0))
            stats[k] = (n + int(r["Calls"]), tot + float(r["TotalDurationNs"]))
pmc = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = defaultdict(lambda: [0.0, 0])
    for f in glob.glob(f"gpurun_out/pin_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != c:
                continue
            k = short(r.get("Kernel_Name", ""))
            if k:
                acc[k][0] += float(r["Counter_Value"]) * 1024.0
                acc[k][1] += 1
    pmc[c] = {k: v[0] / max(v[1], 1) for k, v in acc.items()}
print(f"{'kernel':22s} {'calls':>6s} {'avg_us':>8s} {'read_MB':>8s} {'write_MB':>8s} {'GB/s':>8s} {'frac':>6s}")
for k in KERNELS:
    if k not in stats:
        continue
    n, tot = stats[k]
    avg = tot / n / 1e3
    rd = pmc["FETCH_SIZE"].get(k, 0.0) * 2.0
    wr = pmc["WRITE_SIZE"].get(k, 0.0)
    gbs = (rd + wr) / (avg * 1e-6) / 1e9 if avg > 0 else 0.0
    print(f"{k:22s} {n:6d} {avg:8.2f} {rd / 1e6:8.2f} {wr / 1e6:8.2f} {gbs:8.1f} {gbs / 8000:6.3f}")
