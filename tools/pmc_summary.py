"""Summarize rocprofv3 --pmc CSV outputs: median per kernel (name filter) of each counter over dispatches.
usage: python tools/pmc_summary.py <dir-prefix> <kernel-substring>"""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def main(prefix, filt):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(prefix + "*/**/*counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if filt not in k:
                continue
            vals[k[:70]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            # per dispatch the CSV holds one row per counter (summed over dimensions by rocprofv3)
            print(f"   {c:28s} median {statistics.median(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
