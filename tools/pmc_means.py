"""Mean of every counter per kernel from a rocprofv3 --pmc counter_collection.csv (one pass):
python tools/pmc_means.py <csv> [name-regex]; per-wave values divide by SQ_WAVES when present."""
import collections, csv, re, sys

filt = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"])[:70]
    if filt and not filt.search(k):
        continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    waves = m.get("SQ_WAVES") or 0
    print(k)
    for c, v in sorted(m.items()):
        per = f"  per wave {v / waves:12.1f}" if waves and c.startswith("SQ_") and c != "SQ_WAVES" else ""
        print(f"   {c:28s} {v:16.1f}{per}")
