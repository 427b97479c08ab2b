"""FETCH_SIZE / WRITE_SIZE calibration (MI355X_MICROARCH.md §HBM: "calibrate on a known byte
count in your own access pattern"): tools/pmc_calib.hip streams 1 GiB per kernel with one access
width; this divides the counters of its two rocprofv3 --pmc passes (committed under
profiles/pmc_calib/) by that byte count and writes profiles/pmc_calibration.json, the factors
bench.py applies to the PMC traffic of its roofline kernel.

GPU box (one pass per counter):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/f -o run -- tools/_bin/pmc_calib
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/w -o run -- tools/_bin/pmc_calib
Usage: python scripts/pmc_calibrate.py
"""
from __future__ import annotations

import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.join(ROOT, "profiles", "pmc_calib")
KNOWN = 1 << 30  # bytes streamed by every calibration kernel
WIDTH = {"unsigned long": 8, "unsigned int": 4, "unsigned char": 1}


def main():
    out = {"source": "tools/pmc_calib.hip, rocprofv3 --pmc passes in profiles/pmc_calib/",
           "known_bytes": KNOWN, "read": {}, "write": {}}
    for fn, counter, kind, kern in (("fetch_size.csv", "FETCH_SIZE", "read", "calib_read"),
                                    ("write_size.csv", "WRITE_SIZE", "write", "calib_write")):
        for r in csv.DictReader(open(os.path.join(D, fn))):
            name = r["Kernel_Name"]
            if r["Counter_Name"] != counter:
                continue
            if kern + "16(" in name:  # the uint4 kernels
                width = 16
            elif kern + "<" in name:
                width = WIDTH[name.split("<", 1)[1].split(">", 1)[0]]
            else:
                continue
            # counter bytes (KB x 1024) per true byte for this access width per lane
            f = round(float(r["Counter_Value"]) * 1024 / KNOWN, 4)
            out[kind][f"{width}B_per_lane"] = f or None  # 0: no usable reading
    out["note"] = ("round 1 read FETCH_SIZE 0 for the 1-B loads: the kernel compared its byte "
                   "XOR against a literal above 255, so the compiler deleted the load loop; the "
                   "comparison value is now a kernel argument (tools/pmc_calib.hip)")
    path = os.path.join(ROOT, "profiles", "pmc_calibration.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
