"""Compacts rocprofv3 --pmc counter_collection CSVs in place to one row per (kernel, counter):
Kernel_Name, Counter_Name, Counter_Value (mean per dispatch), Dispatches.  bench.py's readers
(mean over a kernel's rows) and scripts/summarize_profiles.py read both layouts; the compact one
keeps each round's committed passes a few KB instead of megabytes (per-dispatch rows churned
~40 k lines per refresh).  Usage: python3 scripts/pmc_compact.py <pmc dir>..."""
import collections
import csv
import os
import sys

FILES = ("fetch_size.csv", "write_size.csv", "sq_counters.csv", "stall.csv")


def compact(path):
    rows = list(csv.DictReader(open(path)))
    if not rows or "Dispatches" in rows[0]:
        return
    sums = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in rows:
        k = (r["Kernel_Name"], r["Counter_Name"])
        sums[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "Dispatches"])
        for k in sorted(sums):
            n = len(disp[k])
            w.writerow([k[0], k[1], repr(sums[k] / n), n])


if __name__ == "__main__":
    for d in sys.argv[1:]:
        for fn in FILES:
            p = os.path.join(d, fn)
            if os.path.exists(p):
                compact(p)
