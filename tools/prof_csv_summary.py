"""Summarise a rocprofv3 --stats kernel_stats.csv per training step: kernel, calls, ms/step, avg us, share."""
import csv
import sys


def main(path, steps, top=25):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':80s} {'calls':>6s} {'ms/step':>8s} {'avg_us':>9s} {'pct':>6s}")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{r['Name'][:80]:80s} {int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e6 / steps:8.2f} "
              f"{float(r['AverageNs']) / 1e3:9.1f} {float(r['Percentage']):6.2f}")
    print(f"total kernel time per step: {tot / 1e6 / steps:.2f} ms ({steps} steps incl. warmup)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 25)
