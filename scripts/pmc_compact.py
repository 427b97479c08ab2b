"""Compacts rocprofv3 --pmc counter_collection CSVs in place to one row per (kernel, counter):
Kernel_Name, Counter_Name, Counter_Value (mean per dispatch), Dispatches.  bench.py's readers
(mean over a kernel's rows) and scripts/summarize_profiles.py read both layouts; the compact one
keeps each round's committed passes a few KB instead of megabytes (per-dispatch rows churned
~40 k lines per refresh).  It also writes <pmc dir>/meta.json: the source hash of the library
the passes profiled (_lib/liborbx.srchash, or $ORBX_LIB_DIR's) and the kernel instances they
hold, which bench.py's readers require to match the library and the stage they report
(bench.pmc_binding).  Usage: python3 scripts/pmc_compact.py <pmc dir>..."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

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


def write_meta(d):
    from bench import kernel_instance
    lib_dir = os.environ.get("ORBX_LIB_DIR") or os.path.join(ROOT, "ar_orbslam2_amd", "_lib")
    with open(os.path.join(lib_dir, "liborbx.srchash")) as f:
        srchash = f.read().strip()
    kernels = set()
    for fn in FILES:
        p = os.path.join(d, fn)
        if os.path.exists(p):
            kernels |= {kernel_instance(r["Kernel_Name"]) for r in csv.DictReader(open(p))}
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump({"lib_srchash": srchash, "experiment_build": bool(os.environ.get("ORBX_LIB_DIR")),
                   "kernels": sorted(kernels)}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    for d in sys.argv[1:]:
        for fn in FILES:
            p = os.path.join(d, fn)
            if os.path.exists(p):
                compact(p)
        write_meta(d)
