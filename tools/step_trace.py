"""One step's kernel sequence from a rocprofv3 --kernel-trace CSV: the kernels between the last two
launches of a marker kernel (default gru_fwd_kernel), with duration, grid and workgroup sizes —
to attribute framework glue (adds, cats, copies, fills) to the tensors it moves.
python tools/step_trace.py TRACE.csv [--marker NAME] > out.txt"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="gru_fwd_kernel")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
if len(idx) < 2:
    raise SystemExit(f"marker {a.marker} seen {len(idx)} times")
lo, hi = idx[-2], idx[-1]
t0 = int(rows[lo]["Start_Timestamp"])
tot = 0.0
print(f"kernels {hi - lo}, span {(int(rows[hi]['Start_Timestamp']) - t0) / 1e3:.1f} us")
print("  start_us    dur_us      grid  wg  kernel")
for r in rows[lo:hi]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].split("(")[0][:110]
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:10.1f} {d:9.2f} {int(r['Grid_Size_X']):9d} "
          f"{int(r['Workgroup_Size_X']):3d}  {name}")
print(f"sum of kernel durations {tot:.1f} us")
