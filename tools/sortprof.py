"""Per-kernel durations and the back-to-back timeline of the last rs_sort_ids call from a
rocprofv3 (>= 7.x) sqlite results file: python tools/sortprof.py <results.db> [n_last]."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for cnt, avg, name in c.execute("select count(*), avg(duration)/1000.0, name from kernels "
                                "group by name order by 2 desc"):
    print(f"{cnt:6d} {avg:9.2f}  {name[:100]}")
ks = c.execute("select name, start, end from kernels order by start").fetchall()[-n_last:]
t0 = ks[0][1]
print("timeline (us from first): start, duration, kernel")
for n, s, e in ks:
    print(f"{(s - t0) / 1e3:8.2f} {(e - s) / 1e3:8.2f}  {n[:70]}")
print("span", round((ks[-1][2] - t0) / 1e3, 2))
