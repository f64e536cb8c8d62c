"""Per-kernel summary of a rocprofv3 --pmc counter_collection.csv (SQ counters of one pass):
calls, mean duration (dispatch timestamps), VGPRs / LDS bytes per workgroup (occupancy), MFMA
busy fraction (SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles: over 1024 SIMDs x GRBM_GUI_ACTIVE / 8
per XCD), the wave-cycle shares spent waiting (SQ_WAIT_INST_ANY, SQ_WAIT_ANY over SQ_WAVE_CYCLES,
all quad-cycles) and VALU instructions per wave.
usage: python tools/pmc_summary.py <counter_collection.csv> [name-regex]"""
import collections
import csv
import re
import sys

path = sys.argv[1]
filt = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
res = {}
for r in csv.DictReader(open(path)):
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", r["Kernel_Name"])
    k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
    if filt and not filt.search(k):
        continue
    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    res[k] = (r.get("VGPR_Count", "?"), r.get("Accum_VGPR_Count", "?"), r.get("LDS_Block_Size", "?"))


def share(v, c):
    return v.get(c, float("nan")) / v["SQ_WAVE_CYCLES"] if v.get("SQ_WAVE_CYCLES") else float("nan")


print(f"{'kernel':44s} {'calls':>5s} {'avg_us':>8s} {'vgpr':>5s} {'agpr':>5s} {'lds':>6s} "
      f"{'mfma':>6s} {'w_inst':>6s} {'w_any':>6s} {'valu/wave':>9s}")
for k in sorted(vals, key=lambda k: -sum(dur[k].values())):
    v = {c: sum(x) / len(x) for c, x in vals[k].items()}
    us = sum(dur[k].values()) / max(len(dur[k]), 1)
    g = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (g * 1024) if g else float("nan")
    vw = v.get("SQ_ACTIVE_INST_VALU", 0.0) / v["SQ_WAVES"] if v.get("SQ_WAVES") else float("nan")
    vg, ag, lds = res[k]
    print(f"{k[:44]:44s} {len(dur[k]):5d} {us:8.1f} {vg:>5s} {ag:>5s} {lds:>6s} {mf:6.3f} "
          f"{share(v, 'SQ_WAIT_INST_ANY'):6.3f} {share(v, 'SQ_WAIT_ANY'):6.3f} {vw:9.0f}")
