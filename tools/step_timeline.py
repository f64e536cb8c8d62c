"""Print one DLRM step's kernel timeline from a rocprofv3 kernel_trace.csv (queue, start, dur)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "inter_fwd_mfma"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 4
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
busy = {}
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy[r["Queue_Id"]] = busy.get(r["Queue_Id"], 0) + (e - s) / 1e3
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:100]}")
print("step span", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3, "busy", {k: round(v, 1) for k, v in busy.items()})
