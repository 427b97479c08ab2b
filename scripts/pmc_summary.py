"""Summarise rocprofv3 --pmc / --kernel-trace CSVs of a bench run: per kernel, average per
dispatch of every counter, plus VALU-busy estimate (wave64 VALU op = 4 SIMD cycles)."""
import collections
import csv
import sys


def load(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        if "orbx" in k:
            d[k.split("::")[-1]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in d.items()}


if __name__ == "__main__":
    # usage: pmc_summary.py <pmc dir: sq_counters.csv, fetch_size.csv, write_size.csv>
    #                       <rocprofv3 kernel_stats.csv of the same command>
    base, stats = sys.argv[1], sys.argv[2]
    sq = load(f"{base}/sq_counters.csv")
    fe = load(f"{base}/fetch_size.csv")
    wr = load(f"{base}/write_size.csv")
    dur = {}
    for r in csv.DictReader(open(stats)):
        dur[r["Name"].split("(")[0].split("::")[-1]] = float(r["AverageNs"]) / 1e3
    print(f"{'kernel':16s} {'us':>7s} {'waves':>7s} {'valu/w':>7s} {'salu/w':>7s} {'lds/w':>6s} "
          f"{'wait%':>5s} {'valu_us':>7s} {'fetchMB':>8s} {'writeMB':>8s}")
    for k, a in sorted(sq.items(), key=lambda kv: -dur.get(kv[0], 0)):
        w = a.get("SQ_WAVES", 1)
        valu_us = a["SQ_INSTS_VALU"] * 4 / 1024 / 2.4e3
        print(f"{k:16s} {dur.get(k, 0):7.1f} {w:7.0f} {a['SQ_INSTS_VALU'] / w:7.0f} "
              f"{a.get('SQ_INSTS_SALU', 0) / w:7.0f} {a.get('SQ_INSTS_LDS', 0) / w:6.0f} "
              f"{100 * a['SQ_WAIT_ANY'] / max(a['SQ_WAVE_CYCLES'], 1):5.0f} {valu_us:7.1f} "
              f"{fe.get(k, {}).get('FETCH_SIZE', 0) / 1024:8.1f} "
              f"{wr.get(k, {}).get('WRITE_SIZE', 0) / 1024:8.1f}")
