"""Where the compute queue waits on the host: rocprofv3 --kernel-trace --hip-trace of a few train steps.

    python tools/host_gaps.py <dir with run_kernel_trace.csv and run_hip_api_trace.csv> [steps=3] [skip=3]

For the last `steps` complete steps (delimited by the fused AdamW launch) it lists every compute-queue
gap longer than 20 us together with the HIP API calls that were in flight on the host during the gap
(the calls that kept the host from enqueueing the next kernel), and sums the host API time per
function over the steps (long synchronous calls: hipMemcpy from pageable memory, hipHostMalloc,
stream / event synchronisation, hipMalloc / hipFree from the caching allocator)."""
import csv
import os
import sys
from collections import defaultdict


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 3  # trailing AdamW launches: the probe-phase steps
    kt = [r for r in load(os.path.join(d, "run_kernel_trace.csv")) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    for r in kt:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    kt.sort(key=lambda r: r["s"])
    ad = [i for i, r in enumerate(kt) if "adamw" in r["Kernel_Name"]]
    if len(ad) < steps + skip + 1:
        raise SystemExit("not enough steps in the trace")
    a, b = ad[-steps - skip], ad[-skip]
    q0 = kt[b]["Queue_Id"]
    comp = [r for r in kt[a:b + 1] if r["Queue_Id"] == q0]
    t_lo, t_hi = comp[0]["e"], comp[-1]["e"]
    api = load(os.path.join(d, "run_hip_api_trace.csv"))
    calls = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e >= t_lo and s <= t_hi:
            calls.append((s, e, r.get("Function") or r.get("Operation") or r.get("Name", "?")))
    calls.sort()
    per = defaultdict(lambda: [0, 0.0, 0.0])
    for s, e, f in calls:
        p = per[f]
        p[0] += 1
        p[1] += (e - s) / 1e3
        p[2] = max(p[2], (e - s) / 1e3)
    span = (t_hi - t_lo) / 1e3
    print(f"{steps} steps, compute-queue span {span:.1f} us ({span / steps:.1f} per step)")
    prev = comp[0]
    tot = 0.0
    for r in comp[1:]:
        gap = (r["s"] - prev["e"]) / 1e3
        if gap > 20:
            tot += gap
            inflight = [(f, (e - s) / 1e3) for s, e, f in calls if s < r["s"] and e > prev["e"] and (e - s) > 10e3]
            print(f"gap {gap:8.1f} us after {prev['Kernel_Name'][:40]:40s} before {r['Kernel_Name'][:40]:40s} "
                  f"host calls >10us in flight: {inflight[:6]}")
        prev = r
    print(f"gaps > 20 us: {tot:.1f} us total ({tot / steps:.1f} per step)")
    print("\nhost HIP API time per step (top 20 by total): calls, total us, max us")
    for f, (n, t, mx) in sorted(per.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"  {f:40s} {n / steps:8.1f} {t / steps:10.1f} {mx:10.1f}")


if __name__ == "__main__":
    main()
