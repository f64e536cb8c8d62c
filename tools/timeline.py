"""Per-step timeline of a rocprofv3 kernel trace of bench.py: steps are delimited by the
interaction forward kernel; prints each kernel of one step (stream, start offset, duration)
and per-stream busy time."""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    if n.startswith("Cijk"):
        m = re.search(r"Cijk_(\w+?)_S_B.*?MT(\d+x\d+x\d+)", n)
        return "GEMM " + (m.group(1) + " " + m.group(2) if m else n[:40])
    return n.replace("void ", "")[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[3] if len(sys.argv) > 3 else "inter_fwd"
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
step = int(sys.argv[2]) if len(sys.argv) > 2 else -2
a, b = starts[step], starts[step + 1]
# include the bottom-MLP kernels before the interaction: start from the previous step's last
t_first = int(rows[a]["Start_Timestamp"])
back = int(sys.argv[4]) if len(sys.argv) > 4 else 12
seg = rows[a - back:b - back] if a >= back else rows[a:b]
t0 = int(seg[0]["Start_Timestamp"])
busy = {}
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r["Queue_Id"]
    busy[q] = busy.get(q, 0) + (e - s)
    print(f"q{q:>2} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {short(r['Kernel_Name'])}")
span = int(seg[-1]["End_Timestamp"]) - t0
print("span us", span / 1e3, {k: v / 1e3 for k, v in busy.items()})
print("step-to-step us", (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
