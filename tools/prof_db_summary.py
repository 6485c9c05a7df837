"""Summarise a rocprofv3 .db (kernel dispatches): per-kernel count, total/avg/min/max us, share."""
import sqlite3
import sys
from collections import defaultdict


def main(path, top=40):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    sym = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    names = {r[0]: r[1] for r in c.execute(f"select id, kernel_name from {sym}")}
    agg = defaultdict(list)
    for kid, s, e in c.execute(f"select kernel_id, start, end from {disp}"):
        agg[names.get(kid, str(kid))].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'kernel':90s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>8s} {'max_us':>8s} {'pct':>6s}")
    for k, v in rows[:top]:
        print(f"{k[:90]:90s} {len(v):6d} {sum(v):10.1f} {sum(v)/len(v):9.2f} {min(v):8.2f} {max(v):8.2f} "
              f"{100*sum(v)/tot:6.2f}")
    print(f"total kernel time {tot/1e3:.2f} ms over {sum(len(v) for v in agg.values())} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
