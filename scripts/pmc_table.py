"""Per-kernel average of every counter collected by scripts/pmc_passes.sh (p*/ dirs)."""
import collections
import csv
import glob
import sys

base = sys.argv[1]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(f"{base}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(d.items()):
    a = {c: sum(v) / len(v) for c, v in cs.items()}
    w = max(a.get("SQ_WAVES", 1), 1)
    print(k)
    for c in sorted(a):
        print(f"   {c:24s} {a[c]:16.0f}  per wave {a[c] / w:12.1f}")
