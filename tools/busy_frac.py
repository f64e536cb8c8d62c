"""GPU busy fraction of the last two thirds of a rocprofv3 kernel trace (host-bound check):
python tools/busy_frac.py gpurun_out/prof_esmm/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seg = rows[len(rows) // 3:]
t0, t1 = int(seg[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in seg)
busy, end = 0, t0
for r in seg:  # union of kernel intervals (side streams overlap)
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if b > end:
        busy += b - max(a, end)
        end = b
print(sys.argv[1], "busy frac", round(busy / (t1 - t0), 3), "kernels", len(seg))
