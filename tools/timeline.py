"""Two-stream accounting of a training step from a rocprofv3 --kernel-trace CSV.

    python tools/timeline.py <run_kernel_trace.csv> [steps_to_use] [trailing_steps_to_skip=2]

Steps are delimited by the fused AdamW launch (the last kernel of a step). For the last
`steps_to_use` complete steps it reports, per HIP queue: kernel time, busy time (union of
intervals), idle gaps; for the compute queue (the one that runs AdamW): its kernels grouped by
name with their time alone on the chip vs. time overlapped by the other queue's kernels, and the
gaps where the compute queue had nothing running (waiting on an event of the other queue, or on
the host). The compute queue's busy + gap time IS the step, so this is the critical-path split
the summary's summed ms/step column cannot give.
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("fer::", "")
    for cut in ("(", "<"):
        i = n.find(cut)
        if cut == "<" and i > 0:
            j = n.find(">", i)
            tmpl = n[i:j + 1] if j > 0 else ""
            n = n[:i] + tmpl
            break
        if i > 0:
            n = n[:i]
    return n[:70]


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def overlap(s, e, others):
    """ns of [s, e) covered by the union of `others` (sorted, merged intervals)."""
    t = 0
    for os_, oe in others:
        if oe <= s:
            continue
        if os_ >= e:
            break
        t += min(e, oe) - max(s, os_)
    return t


def merged(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def main(path, nsteps=5, skip_tail=2):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"]))
    rows.sort()
    ends = [e for s, e, q, n in rows if "adamw_kernel" in n]
    if len(ends) - skip_tail < nsteps + 1:
        nsteps = len(ends) - skip_tail - 1
    # the last `skip_tail` steps are bench.py's probe phase (weight gradients on the compute stream)
    ends = ends[:len(ends) - skip_tail] if skip_tail else ends
    t0, t1 = ends[-nsteps - 1], ends[-1]
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    cq = [q for s, e, q, n in win if "adamw_kernel" in n][0]
    queues = sorted({q for _, _, q, _ in win})
    span = (t1 - t0) / nsteps
    print(f"steps {nsteps}, step {span / 1e6:.3f} ms (AdamW end to AdamW end); compute queue {cq}")
    per_q = {q: [(s, e) for s, e, qq, _ in win if qq == q] for q in queues}
    for q in queues:
        k = sum(e - s for s, e in per_q[q]) / nsteps
        b = union(per_q[q]) / nsteps
        print(f"queue {q}{' (compute)' if q == cq else ''}: {len(per_q[q]) // nsteps} kernels/step, kernel time "
              f"{k / 1e6:.3f} ms, busy {b / 1e6:.3f} ms, idle {(span - b) / 1e6:.3f} ms per step")
    other = merged([(s, e) for s, e, q, _ in win if q != cq])
    by = defaultdict(lambda: [0, 0, 0])
    for s, e, q, n in win:
        if q != cq:
            continue
        d = by[short(n)]
        d[0] += 1
        d[1] += e - s
        d[2] += overlap(s, e, other)
    print(f"\ncompute-queue kernels (per step): calls, ms, of which overlapped by the other queue(s), mean us")
    print(f"{'kernel':70s} {'calls':>5s} {'ms':>7s} {'ovl ms':>7s} {'alone ms':>8s} {'mean us':>8s}")
    tot = [0, 0]
    for n, (c, t, o) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        tot[0] += t
        tot[1] += o
        print(f"{n:70s} {c // nsteps:5d} {t / nsteps / 1e6:7.3f} {o / nsteps / 1e6:7.3f} {(t - o) / nsteps / 1e6:8.3f} "
              f"{t / c / 1e3:8.1f}")
    print(f"{'total':70s} {'':5s} {tot[0] / nsteps / 1e6:7.3f} {tot[1] / nsteps / 1e6:7.3f} "
          f"{(tot[0] - tot[1]) / nsteps / 1e6:8.3f}")
    oby = defaultdict(lambda: [0, 0])
    for s, e, q, n in win:
        if q == cq:
            continue
        d = oby[short(n)]
        d[0] += 1
        d[1] += e - s
    print("\nother-queue kernels (per step)")
    for n, (c, t) in sorted(oby.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:70s} {c // nsteps:5d} {t / nsteps / 1e6:7.3f} {t / c / 1e3:8.1f}")
    # compute-queue gaps: nothing running on the compute queue
    cint = merged(per_q[cq])
    gaps = []
    for (s0, e0), (s1, e1) in zip(cint, cint[1:]):
        if s1 - e0 > 0:
            gaps.append((s1 - e0, e0))
    g_all = sum(g for g, _ in gaps)
    g_big = [g for g in gaps if g[0] > 20000]
    print(f"\ncompute-queue gaps: {g_all / nsteps / 1e6:.3f} ms/step total, {len(gaps) // nsteps} per step; "
          f"{len(g_big) / nsteps:.1f} per step longer than 20 us ({sum(g for g, _ in g_big) / nsteps / 1e6:.3f} ms)")
    # what the compute queue launched right after its longest gaps
    starts = {e: None for _, e in gaps}
    nxt = {}
    for g, e0 in sorted(gaps, reverse=True)[:8]:
        after = [r for r in win if r[2] == cq and r[0] >= e0]
        nxt[e0] = short(after[0][3]) if after else "?"
        print(f"  gap {g / 1e3:8.1f} us before {nxt[e0]}")
    # tail: time between the compute queue's last backward kernel and the AdamW launch of each step
    del starts


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5, int(sys.argv[3]) if len(sys.argv) > 3 else 2)
