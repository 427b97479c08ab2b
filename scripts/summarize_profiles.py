"""Summaries of the committed round evidence under profiles/ (written by
scripts/refresh_profiles.sh):

  <tag>_roofline_check.txt  per config: the bench line's roofline kernel, its average launch
                            duration from bench.py's HIP events (roofline pass, camera stream 0
                            alone) against the rocprofv3 kernel trace of the same command
                            (all dispatches: timed region with 3 concurrent streams + roofline
                            pass; last 5 dispatches: the roofline pass itself)
  <tag>_pmc_summary.txt     per config and kernel: trace average, waves, VALU / SALU / LDS
                            instructions per wave, SQ_WAIT_ANY share, VALU issue floor and the
                            FETCH_SIZE / WRITE_SIZE megabytes per dispatch

Usage: python scripts/summarize_profiles.py [r01]
"""
from __future__ import annotations

import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
# config -> (suffix of the bench / kernel stats / trace files, suffix of the PMC dir)
CONFIGS = {"C2": ("", ""), "AR": ("_ar", "_ar"), "C3": ("_c3", "_c3"), "C4": ("_c4", "_c4"),
           "C5": ("_c5", "_c5")}
QC_US = 4 / (1024 * 2.4e3)  # us per SIMD quad-cycle of issue (1024 SIMDs, 2.4 GHz)


def short(name: str) -> str:
    for ns in ("void ", "orbx::cvorb::", "orbx::", "(anonymous namespace)::"):
        name = name.replace(ns, "")
    return name.split("(")[0]


def trace_durations(path):
    """kernel -> [(duration ns, stream id, solo)] in dispatch-time order; `solo`: no dispatch of
    another stream (any kernel) overlaps it in time"""
    d = collections.defaultdict(list)
    allr = []
    with open(path) as f:
        for r in csv.DictReader(f):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            st = r.get("Stream_Id", "")
            allr.append((t0, t1, st))
            d[short(r["Kernel_Name"])].append((t0, t1, st))
    allr.sort()
    starts = [a[0] for a in allr]

    def solo(t0, t1, st):
        # dispatches starting before t1; any of another stream still running after t0 overlaps
        import bisect
        k = bisect.bisect_left(starts, t1)
        for a0, a1, ast in allr[max(0, k - 64):k]:
            if ast != st and a1 > t0:
                return False
        return True

    return {k: [(t1 - t0, st, solo(t0, t1, st)) for t0, t1, st in sorted(v)] for k, v in d.items()}


def solo_run(d, steps=5):
    """The roofline pass's dispatches: stream 0 alone after the timed region, so the longest run
    of consecutive dispatches on one stream that no other stream's dispatch overlaps (the timed
    region before it and the PCIe pass after it run the camera streams concurrently)."""
    best, i = [], 0
    while i < len(d):
        j = i
        while j < len(d) and d[j][1] == d[i][1] and d[j][2]:
            j += 1
        if j - i >= steps and j - i > len(best):
            best = [x[0] for x in d[i:j]]
        i = max(j, i + 1)
    return best[:steps] or [x[0] for x in d[-steps:]]


def counters(pmc_dir):
    """kernel -> counter -> sum over dispatches, and (kernel, counter) -> dispatches; reads the
    per-dispatch rocprofv3 layout and the compact one of scripts/pmc_compact.py"""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    counts = collections.Counter()
    for fn in ("fetch_size.csv", "write_size.csv", "sq_counters.csv"):
        path = os.path.join(pmc_dir, fn)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                if "Dispatches" in r:  # compact: mean per dispatch of one full kernel name
                    n = int(r["Dispatches"])
                    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]) * n
                    counts[(k, r["Counter_Name"])] += n
                else:
                    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    ids[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    calls = {key: range(counts[key] + len(ids.get(key, ()))) for key in set(counts) | set(ids)}
    return agg, calls


def main(tag="r02"):
    check, summ = [], []
    for cfg, (sfx, psfx) in CONFIGS.items():
        bench = os.path.join(P, f"{tag}_bench{sfx}.jsonl")
        trace = os.path.join(P, "traces", f"{tag}_kernel_trace{sfx}.csv")
        if not os.path.exists(trace):  # round 3 on: traces stay in gpurun_out (not committed)
            trace = os.path.join(ROOT, "gpurun_out", tag, "traces", f"kernel_trace{sfx}.csv")
        if not os.path.exists(trace) and tag == "r01":  # round-1 layout
            trace = os.path.join(P, "traces", f"kernel_trace{sfx}.csv")
        if not (os.path.exists(bench) and os.path.exists(trace)):
            continue
        line = json.loads(open(bench).read().strip().splitlines()[-1])
        rf = line["roofline"]
        durs = trace_durations(trace)
        k = rf["kernel"]
        # every instance of the kernel (k_fast_cells runs a <44, 44> and a <72, 66> launch per
        # step; bench.py's stage, one "launch", spans both): durations summed per step
        # (and k_fast_pairs, the pair kernel of the same stage)
        names = {"k_fast_cells": ("k_fast_cells", "k_fast_pairs")}.get(k, (k,))
        inst = [v for kk, v in sorted(durs.items())
                if any(kk == nm or kk.startswith(nm + "<") for nm in names)]
        check.append(f"{cfg} ({line['config']['workload']}): {line['value']:.1f} frames/s")
        check.append(f"  kernel {k}: {sum(len(v) for v in inst)} dispatches"
                     + (f" ({len(inst)} instances, summed per step)" if len(inst) > 1 else ""))
        if inst:
            # a stage with several dispatches per step (k_pyramid: one per pyramid stage) is
            # averaged per dispatch, as bench.py's avg_launch_us
            lps = int(round(rf.get("launches_per_step", 1) or 1))
            solo = [sum(x) for x in zip(*(solo_run(v, 5 * lps) for v in inst))]
            alld = sum(sum(x[0] for x in v) / len(v) for v in inst)
            check.append(f"    trace average, all dispatches (timed region with concurrent streams"
                         f" + roofline pass + PCIe pass): {alld / 1e3:.2f} us")
            check.append(f"    trace average, roofline pass ({len(solo)} consecutive dispatches on one "
                         f"stream, camera stream 0 alone): {sum(solo) / len(solo) / 1e3:.2f} us")
        under = os.path.join(P, f"{tag}_bench{sfx}_under_rocprof.jsonl")
        if os.path.exists(under):
            ru = json.loads(open(under).read().strip().splitlines()[-1])["roofline"]
            check.append(f"    bench.py roofline avg_launch_us of the traced run (HIP events, same "
                         f"pass): {ru['avg_launch_us']:.2f} us")
        check.append(f"    bench.py roofline avg_launch_us of the committed line (separate run): "
                     f"{rf['avg_launch_us']:.2f} us")
        vr = rf.get("issue_roofline") or rf.get("valu_roofline") or {}
        hb = rf.get("hbm") or rf
        check.append(f"    HBM: achieved {hb.get('achieved')} GB/s of {hb.get('peak')} (frac "
                     f"{hb.get('frac')}); issue floors: VALU {vr.get('valu_floor_us')} us, SALU "
                     f"{vr.get('salu_floor_us')} us, bound {vr.get('issue_bound')} (frac "
                     f"{vr.get('frac')})")
        agg, calls = counters(os.path.join(P, f"{tag}_pmc{psfx}"))
        summ.append(f"# {cfg}: per dispatch; us = rocprofv3 trace average of the bench command "
                    f"(3 concurrent streams + roofline pass)")
        summ.append("# valu_us / salu_us: issue floors per dispatch, (ACTIVE_INST_VALU - "
                    "ACTIVE_INST_VALU2) x 4 and INSTS_SALU x 4 cycles over 1024 SIMDs at 2.4 GHz")
        summ.append(f"{'kernel':28s}{'us':>9s}{'waves':>9s}{'valu/w':>8s}{'salu/w':>8s}"
                    f"{'lds/w':>7s}{'wait%':>6s}{'valu_us':>9s}{'salu_us':>9s}{'fetchMB':>9s}"
                    f"{'writeMB':>9s}")
        rows = []
        for kn, dd in ((kn, [x[0] for x in v]) for kn, v in durs.items()):
            a = agg.get(kn, {})

            def per(c):
                n = len(calls.get((kn, c), ())) or 1
                return a.get(c, 0.0) / n
            w = per("SQ_WAVES") or 1.0
            cyc = per("SQ_WAVE_CYCLES") or 1.0
            qc = (per("SQ_ACTIVE_INST_VALU") - per("SQ_ACTIVE_INST_VALU2")
                  if "SQ_ACTIVE_INST_VALU2" in a else per("SQ_INSTS_VALU"))
            rows.append((sum(dd) / len(dd) / 1e3, kn, per("SQ_WAVES"), per("SQ_INSTS_VALU") / w,
                         per("SQ_INSTS_SALU") / w, per("SQ_INSTS_LDS") / w,
                         100 * per("SQ_WAIT_ANY") / cyc, qc * QC_US, per("SQ_INSTS_SALU") * QC_US,
                         per("FETCH_SIZE") / 1024, per("WRITE_SIZE") / 1024))
        for r in sorted(rows, reverse=True):
            if r[1].startswith("__amd"):
                continue
            summ.append(f"{r[1][:27]:28s}{r[0]:9.1f}{r[2]:9.0f}{r[3]:8.0f}{r[4]:8.0f}{r[5]:7.0f}"
                        f"{r[6]:6.0f}{r[7]:9.1f}{r[8]:9.1f}{r[9]:9.1f}{r[10]:9.1f}")
        # k_describe: counter traffic per keypoint against the bytes one keypoint's 37x37 blurred
        # patch holds (the image pyramid is read once per image at batch 512, so the traffic is
        # the pyramid's bytes spread over the keypoints, not the patches)
        c = line["config"]
        kp = c.get("keypoints_per_frame", 0) * c.get("frames_per_batch", 0) * c.get("images_per_frame", 1)
        for r in rows:
            if r[1].startswith("k_describe") and kp:
                # FETCH_SIZE reads 1/2 of the bytes loaded (profiles/pmc_calibration.json)
                fb, wb = r[9] * 1024 * 1024 / 0.5 / kp, r[10] * 1024 * 1024 / kp
                pyr = 2 * c.get("frames_per_batch", 0) * c.get("images_per_frame", 1)
                summ.append(f"# k_describe per keypoint ({kp:.0f} keypoints per dispatch): fetched "
                            f"{fb:.0f} B (FETCH_SIZE / 0.5), written {wb:.0f} B; one keypoint's "
                            f"31x31 raw + 37x37 blurred patches 2330 B, algorithmic (keypoint in + "
                            f"descriptor out) 60 B; fetched per dispatch {r[9] / 0.5:.0f} MB for "
                            f"{pyr} pyramids (raw + blurred) of {c.get('frames_per_batch')} images")
        summ.append("")
    open(os.path.join(P, f"{tag}_roofline_check.txt"), "w").write("\n".join(check) + "\n")
    open(os.path.join(P, f"{tag}_pmc_summary.txt"), "w").write("\n".join(summ))
    print("\n".join(check))


if __name__ == "__main__":
    main(*sys.argv[1:])
