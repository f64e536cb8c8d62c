"""Turn a rocprofv3 --stats kernel_stats.csv into the text table committed under profiles/."""
import csv
import sys


def main(src, dst, header):
    rows = list(csv.DictReader(open(src)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    with open(dst, "w") as f:
        f.write(header.rstrip() + "\n\n")
        f.write(f"{'calls':>6} {'total_us':>10} {'avg_us':>9}  kernel\n")
        for r in rows[:40]:
            f.write(f"{int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e3:10.1f} "
                    f"{float(r['AverageNs']) / 1e3:9.1f}  {r['Name'][:150]}\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
