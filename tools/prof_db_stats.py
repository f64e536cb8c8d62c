"""Per-kernel stats (calls, total / average us) from a rocprofv3 results database (the default
rocpd SQLite output, run_results.db), optionally per step: python tools/prof_db_stats.py DB
[--steps N] [--top K]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for name, dur in c.execute("select name, duration from kernels"):
        tot[name] += dur / 1e3
        cnt[name] += 1
    print(f"{'calls/step':>10} {'us/step':>9} {'avg_us':>8}  kernel")
    for name in sorted(tot, key=lambda n: -tot[n])[:a.top]:
        print(f"{cnt[name] / a.steps:10.1f} {tot[name] / a.steps:9.1f} {tot[name] / cnt[name]:8.1f}  "
              f"{name[:110]}")
    print(f"all kernels: {sum(tot.values()) / a.steps:.1f} us/step")


if __name__ == "__main__":
    main()
