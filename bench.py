#!/usr/bin/env python3
"""Benchmark: frames/s of ORB extract + match (BASELINE.json metric) on MI355X.

One step = one batch of `--batch` synthetic 640x480 frames (BASELINE.json configs[1], TUM
fr1/xyz mono geometry, 1000 features) per camera stream, already resident in HBM, pushed
through the whole device pipeline: ORBextractor (pyramid, FAST cells, octree, orientation,
rBRIEF), Frame::ComputeBoW (full DBoW2 descent of the seeded k=10, L=6 vocabulary: word ids,
BowVector, FeatureVector), SearchByBoW(prev-as-KF, cur) and SearchForTriangulation(prev-as-KF,
cur-as-KF) (SURVEY §8d unit of work).

Multi-GPU: one process per GPU.  Camera streams are independent; global stream s
runs on rank s mod G (the reference's only parallelism is one extractor per camera thread,
ORB_SLAM2/src/Frame.cc:83-86), so there is no data-path collective: RCCL carries only the
barrier and the max-over-ranks time.  Weak scaling (default): `--streams` camera streams per
GPU.  Strong scaling: `--streams-total T` fixes the job's stream count over G GPUs.  Under
torchrun the rank comes from RANK / LOCAL_RANK / WORLD_SIZE; `--gpus N` without WORLD_SIZE
starts the N rank processes itself before anything touches the GPU.

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (HIP events on the
pipeline stream), the PCIe-upload-included rate, and the CPU oracle baseline (rank 0, N=1).
`--dropin` measures the per-frame drop-in path instead (tools/orbx_dropin.cpp: host threads
calling orbx_extract / orbx_vocabulary_transform / orbx_search_* one frame at a time).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match, 640×480 1000-feat; bit-exact descriptors"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PCIE_GEN5_X16_GBS = 63.0  # PCIe Gen5 x16 spec, one direction
VALU_SIMDS = 1024         # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4           # MI355X peak engine clock
CONFIGS = {
    # batch: frames per step per camera stream (C2: 3 x 512 measured 225.5k vs 3 x 256 222.3k
    # frames/s, three alternating runs each on one box; C3 / C4: 512 vs 256 107.6-108.1k vs
    # 106.4-106.6k and 71.0-71.3k vs 70.8-71.0k, C5 44.2-44.5k vs 43.7-44.0k, two runs each
    # (scripts/gpu_batch_ab.sh); AR below)
    "C2": dict(w=640, h=480, nfeatures=1000, batch=512,
               workload="TUM fr1/xyz mono 640x480, 1000 features, 1xMI355X HIP extract+match"),
    "C3": dict(w=752, h=480, nfeatures=1200, stereo=(47.90639384423901, 435.2046959714599), batch=512,
               workload="EuRoC MH01 stereo geometry 2x752x480, 1200 features, stereo matching"),
    "C4": dict(w=1241, h=376, nfeatures=2000, stereo=(386.1448, 718.856), batch=512,
               workload="KITTI 00 stereo geometry 2x1241x376, 2000 features, stereo matching"),
    "C5": dict(w=1920, h=1080, nfeatures=4000, batch=512,
               workload="synthetic 1920x1080, 4000 features"),
    # the AR marker path (Marker::Match: cv::ORB 2.4 HARRIS 500 features on
    # the frame, BruteForceMatcher<HammingLUT> against the target's descriptors, good filter)
    # AR: 512 vs 256 frames per batch 282.8-283.1k vs 272.0-275.0k frames/s, two runs each
    "AR": dict(w=640, h=480, nfeatures=500, marker=True, batch=512,
               workload="AR marker path 640x480: cv::ORB (500, HARRIS_SCORE) + BruteForceMatcher "
                        "vs a 500-feature target + Marker::Match filter"),
}
MARKER_METRIC = "frames/sec AR Marker::Match (cv::ORB HARRIS 500 + BF Hamming match), 640x480"


def level_sizes(w, h, inv_scale):
    return [(int(np.rint(np.float32(w) * np.float32(s))), int(np.rint(np.float32(h) * np.float32(s))))
            for s in inv_scale]


def algorithmic_bytes(levels, n_kp, n_img):
    """Per-kernel algorithmic bytes for one launch over n_img images (SURVEY §8d byte model:
    input read, resize read+write, FAST read, blur read+write, 28+32 B per keypoint)."""
    P = [w * h for w, h in levels]
    per_resize = [(P[l - 1] + P[l]) * n_img for l in range(1, len(P))]
    return {
        # per step; a stage's launch is one dispatch (roofline_of divides by the dispatches per
        # step: k_pyramid runs one per pyramid stage).  SURVEY §8d counts the input once (P0
        # read); the kernel also writes level 0 into the pitched pyramid (one more P0), which
        # is reported beside the §8d figure as the builder's model, never used for `frac`
        "k_pyramid": P[0] * n_img + sum(per_resize),
        "k_pyramid_level0_write": P[0] * n_img,
        "k_blur": 2 * sum(P) * n_img,
        # SURVEY §8d's FAST term: every level pixel read once (the per-cell kernel writes only
        # the cells' keys, 4 B per candidate, ~1 % of the pixels: not counted)
        "k_fast_cells": sum(P) * n_img,
        "k_describe": 60 * n_kp,
        "k_voc_transform": 52 * n_kp,                          # desc in; word, rank, node, weight out
        "k_bowvec": 24 * n_kp,
        "total_per_frame": P[0] + sum(per_resize) / n_img + 3 * sum(P) + 60 * n_kp / n_img,
    }


# bytes per lane of the global loads of the kernels bench.py can name as roofline kernel (the
# staged windows of k_cvfast: 16-B pieces per lane; k_fast_cells: the cell ROI as aligned
# dwords; k_pyramid: the source band's 16-B chunks); the stores are 8-B bitmap words (k_cvfast),
# 4-B keys (k_fast_cells) and 4-B pixel groups (k_pyramid)
LOAD_WIDTH = {"k_cvfast": 16, "k_fast_cells": 4, "k_fast_pairs": 4, "k_pyramid": 16}


def _load_json(name):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return None


# The PMC passes of a round (scripts/refresh_profiles.sh): profiles/<PMC_ROUND>_pmc[_<config>]
PMC_ROUND = "r06"


def kernel_instance(name):
    """rocprofv3 Kernel_Name -> the instance name the library's profiler records:
    'void orbx::k_fast_cells<44, 42, unsigned int>(unsigned char const*, ...)' ->
    'k_fast_cells<44, 42, unsigned int>'; 'orbx::k_tri_nodes(...)' -> 'k_tri_nodes'."""
    s = name.replace("(anonymous namespace)::", "")
    if s.startswith("void "):
        s = s[5:]
    depth = 0
    for i, ch in enumerate(s):  # the signature's '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            s = s[:i]
            break
    head, sep, args = s.partition("<")
    return head.split("::")[-1] + sep + args


def library_hash():
    """(source hash recorded by the loaded library's build, whether it is an experiment build
    (ORBX_LIB_DIR + ORBX_ALLOW_CUSTOM_BUILD), its directory)."""
    from ar_orbslam2_amd import _ffi
    return _ffi.source_hash()[1], _ffi.EXPERIMENT_LIB, os.path.dirname(_ffi.LIB_PATH)


def library_info():
    """The library build behind a bench line: its recorded source hash, and whether it is an
    experiment build (ORBX_LIB_DIR + ORBX_ALLOW_CUSTOM_BUILD: not checked against the tree's
    sources, so never evidence for the tree)."""
    built, exp, lib_dir = library_hash()
    return {"srchash": built, "experiment_build": bool(exp),
            "lib_dir": os.path.relpath(lib_dir, ROOT) if exp else None}


def pmc_binding(pmc_dir, instances):
    """Checks that the PMC passes in pmc_dir were collected from the library this process runs
    (meta.json's lib_srchash, written by scripts/pmc_compact.py next to the passes) and hold
    every kernel instance the timed stage launched.  Returns a reason string when they do not
    (the counter fields are then null), else None."""
    rel = os.path.relpath(pmc_dir, ROOT) if pmc_dir else None
    if not pmc_dir or not os.path.isdir(pmc_dir):
        return f"no PMC passes for this command ({rel})"
    try:
        meta = json.load(open(os.path.join(pmc_dir, "meta.json")))
    except (OSError, ValueError):
        return f"PMC passes without meta.json: not bound to a library build ({rel})"
    built, _, _ = library_hash()
    if not built or meta.get("lib_srchash") != built:
        return (f"PMC passes of another library build ({rel}: {meta.get('lib_srchash')}; "
                f"this run: {built})")
    if not instances:
        return "the stage's kernel instances are unknown (no profiled run)"
    have = set(meta.get("kernels", []))
    missing = [k for k in instances if k not in have]
    if missing:
        return f"kernel instance(s) {missing} not in the PMC passes ({rel})"
    return None


def pmc_traffic(pmc_dir, instances, stage=None):
    """HBM-side bytes per launch of a stage (its kernel `instances`, exact rocprofv3 names) from
    separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, both in KB) of the same library
    build (pmc_binding).  MI355X_MICROARCH.md §HBM: FETCH_SIZE counts L2->fabric
    requests (Infinity-Cache hits included) and reads 1/2 of the bytes of 16-B-per-lane streaming
    loads; other widths are to be calibrated in one's own access pattern, which
    profiles/pmc_calibration.json holds (tools/pmc_calib.hip).  Returns (bytes, note):
    FETCH_SIZE x 1024 / read factor of the kernel's load width + WRITE_SIZE x 1024 / the 8-B
    store factor, or the uncorrected sum without a calibration; (None, reason) when the passes
    do not belong to this build or lack one of the instances."""
    import csv
    why = pmc_binding(pmc_dir, instances)
    if why:
        return None, why
    tot = {}
    rel = os.path.relpath(pmc_dir, ROOT)
    for name, counter in (("fetch_size.csv", "FETCH_SIZE"), ("write_size.csv", "WRITE_SIZE")):
        path = os.path.join(pmc_dir, name)
        if not os.path.exists(path):
            return None, f"no {counter} pass ({rel})"
        # one "launch" of a stage spans every instance it launched (k_fast_pairs and the
        # k_fast_cells instances per step): mean per instance over its dispatches, summed
        per = {}
        for r in csv.DictReader(open(path)):
            if kernel_instance(r["Kernel_Name"]) in instances and r["Counter_Name"] == counter:
                per.setdefault(kernel_instance(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
        if set(per) != set(instances):
            return None, f"{counter} lacks {sorted(set(instances) - set(per))} ({rel})"
        tot[counter] = sum(sum(v) / len(v) for v in per.values()) * 1024
    cal = _load_json("pmc_calibration.json")
    # the load width of the stage (its instances may be different kernels: the k_fast_cells
    # stage launches k_fast_pairs first); instances of different widths get no correction
    widths = {LOAD_WIDTH.get(i.split("<")[0]) for i in instances}
    w = LOAD_WIDTH.get(stage) if stage else (widths.pop() if len(widths) == 1 else None)
    if stage and len(widths - {None}) > 1:
        w = None
    rf = (cal or {}).get("read", {}).get(f"{w}B_per_lane") if w else None
    wf = (cal or {}).get("write", {}).get("8B_per_lane")
    if rf and wf:
        return (round(tot["FETCH_SIZE"] / rf + tot["WRITE_SIZE"] / wf),
                f"FETCH_SIZE*1024/{rf} + WRITE_SIZE*1024/{wf} per launch: rocprofv3 --pmc passes of "
                f"this command ({rel}), corrected by profiles/pmc_calibration.json for {w}-B loads")
    return (round(tot["FETCH_SIZE"] + tot["WRITE_SIZE"]),
            f"uncorrected (FETCH_SIZE+WRITE_SIZE)*1024 per launch ({rel}; no calibration for "
            f"this kernel's access width)")


def pmc_issue(pmc_dir, instances, avg_launch_us):
    """Issue-rate roofline of `kernel` from the SQ counter pass of this bench command
    (sq_counters.csv, per-dispatch sums over the chip's SIMDs).  Measured on this MI355X with
    tools/valu_calib.hip (profiles/valu_calibration.json): a wave64 VALU instruction occupies
    its SIMD for one quad-cycle (4 cycles) except 32-bit add / sub / and / or / xor and f32 add /
    fma, which dual-issue (2 cycles: SQ_ACTIVE_INST_VALU2 counts the quad-cycles in which two
    VALU instructions issued), and a SALU instruction takes one quad-cycle of its SIMD's scalar
    issue (SQ_INST_CYCLES_SALU == SQ_INSTS_SALU).  So a launch cannot finish before
      VALU floor = (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) x 4 / (1024 SIMDs x 2.4 GHz)
      SALU floor = SQ_INSTS_SALU x 4 / (1024 SIMDs x 2.4 GHz)
    and the larger floor is the bound.  Older passes without SQ_ACTIVE_INST_VALU2 price every
    VALU instruction at 4 cycles (the calibrated cost of all but the dual-issue ops)."""
    import csv
    why = pmc_binding(pmc_dir, instances)
    path = os.path.join(pmc_dir, "sq_counters.csv") if pmc_dir else ""
    if why or not os.path.exists(path) or not avg_launch_us:
        return {"valu_floor_us": None, "frac": None,
                "note": why or f"no SQ counter pass ({os.path.relpath(path, ROOT) if path else None})"}
    per = {}  # counter -> instance -> values per dispatch
    for r in csv.DictReader(open(path)):
        k = kernel_instance(r["Kernel_Name"])
        if k in instances:
            per.setdefault(r["Counter_Name"], {}).setdefault(k, []).append(float(r["Counter_Value"]))
    if "SQ_INSTS_VALU" not in per or set(per["SQ_INSTS_VALU"]) != set(instances):
        return {"valu_floor_us": None, "frac": None,
                "note": f"the SQ pass lacks an instance of {instances}"}
    # per stage launch: mean per instance, summed over the kernel's instances
    avg = {k: sum(sum(v) / len(v) for v in inst.values()) for k, inst in per.items()}
    us_per_qc = 4 / VALU_SIMDS / (CLOCK_GHZ * 1e3)
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_ACTIVE_INST_VALU2" in avg:
        valu_qc = avg["SQ_ACTIVE_INST_VALU"] - avg["SQ_ACTIVE_INST_VALU2"]
        how = "(SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) quad-cycles"
    else:
        valu_qc = avg["SQ_INSTS_VALU"]
        how = "SQ_INSTS_VALU x 1 quad-cycle (no SQ_ACTIVE_INST_VALU2 in this pass)"
    valu_us = valu_qc * us_per_qc
    salu_us = avg.get("SQ_INSTS_SALU", 0.0) * us_per_qc
    bound = "valu" if valu_us >= salu_us else "salu"
    floor = max(valu_us, salu_us)
    return {"kernels": list(instances), "valu_instr_per_launch": round(avg["SQ_INSTS_VALU"]),
            "valu_quad_cycles_per_launch": round(valu_qc),
            "salu_instr_per_launch": round(avg.get("SQ_INSTS_SALU", 0.0)),
            "valu_floor_us": round(valu_us, 2), "salu_floor_us": round(salu_us, 2),
            "issue_bound": bound, "issue_floor_us": round(floor, 2),
            "frac": round(floor / avg_launch_us, 4),
            "note": f"VALU floor = {how} x 4 cycles / ({VALU_SIMDS} SIMDs x {CLOCK_GHZ} GHz); "
                    f"SALU floor = SQ_INSTS_SALU x 4 cycles / the same; frac = larger floor / "
                    f"avg_launch_us; costs from profiles/valu_calibration.json "
                    f"({os.path.relpath(path, ROOT)})"}


AGGREGATE_STAGES = ("k_stereo", "k_bow", "k_tri")


def roofline_of(stages, alg, pmc_dir, steps, B, kernels=None):
    """Roofline object of the dominant kernel (largest total time in the per-kernel HIP-event
    pass), in the contract's terms: `bound` "hbm", `achieved` = SURVEY §8d's algorithmic bytes
    per launch / the average launch time, `peak` 8 TB/s, `frac` = achieved / peak.  The path is
    integer stencil / gather / popcount work whose binding ceiling is instruction issue, not
    bytes: that roofline (VALU / SALU quad-cycles per launch from the SQ counters of this command
    against the issue rate of 1024 SIMDs) is reported beside it in `issue_roofline`."""
    # stages not launched in this configuration (the other FAST path) are dropped
    stages = {k: v for k, v in stages.items() if v[1] > 0}
    if "k_pyramid" in stages and "k_blur" not in stages and "k_blur" in alg:
        # the blur fused into k_pyramid's bands (Geometry::blur_fused): its read + write of every
        # level (SURVEY §8d's 2 sum(P)) belong to the pyramid's launches
        alg = dict(alg, k_pyramid=alg["k_pyramid"] + alg["k_blur"])
    # stages that time several kernels (the stereo copy + 3 kernels, the matchers' node and
    # finish kernels) cannot be matched to one kernel's counters: the roofline kernel is the
    # largest single-kernel stage
    single = {k: v for k, v in stages.items() if k not in AGGREGATE_STAGES}
    if not single:
        return None
    dom = max(single, key=lambda k: single[k][0])
    ms, launches = stages[dom]
    avg_s = ms / 1e3 / max(launches, 1)
    # algorithmic bytes are per step; a stage with several dispatches per step (k_pyramid: one
    # per pyramid stage) splits them over its launches, as the PMC readers average per dispatch
    per_step = max(launches, 1) / max(steps, 1)
    a_bytes = alg.get(dom) / per_step if alg.get(dom) is not None else None
    achieved = (a_bytes / avg_s / 1e9) if a_bytes is not None else None
    # the kernel instances the roofline pass launched for this stage (the library's profiler):
    # the PMC fields are those instances' counters from passes of this same library build
    inst = (kernels or {}).get(dom) or []
    traffic, tnote = pmc_traffic(pmc_dir, inst, dom)
    issue = pmc_issue(pmc_dir, inst, avg_s * 1e6)
    hbm = {"achieved": round(achieved, 3) if achieved is not None else None,
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 6) if achieved is not None else None}
    out = {"bound": "hbm", "kernel": dom, "kernel_instances": inst, **hbm, "traffic": traffic,
           "traffic_note": tnote,
           "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_bytes_per_launch": a_bytes,
           "algorithmic_bytes_model": "SURVEY §8d",
           "launches_per_step": round(per_step, 3)}
    if dom == "k_pyramid" and alg.get("k_pyramid_level0_write") and a_bytes is not None:
        # the builder's model adds the level-0 write into the pitched pyramid (not a §8d term)
        b_bytes = a_bytes + alg["k_pyramid_level0_write"] / per_step
        out["builder_model"] = {"algorithmic_bytes_per_launch": b_bytes,
                                "extra_term": "level-0 write into the pyramid, P0 per image",
                                "frac": round(b_bytes / avg_s / 1e9 / HBM_PEAK_GBS, 6)}
    if issue and issue.get("frac") is not None:
        # the issue-rate roofline (achieved / peak in SIMD quad-cycles of the binding unit per
        # second)
        qc = (issue["valu_quad_cycles_per_launch"] if issue["issue_bound"] == "valu"
              else issue["salu_instr_per_launch"])
        peak_gqc = VALU_SIMDS * CLOCK_GHZ / 4  # G SIMD quad-cycles per second
        issue = dict(issue, achieved=round(qc / avg_s / 1e9, 3), peak=round(peak_gqc, 3),
                     unit=f"G {issue['issue_bound'].upper()} issue quad-cycles/s")
    out["issue_roofline"] = issue
    out["stages_ms_per_step"] = {k: round(v[0] / steps, 4) for k, v in stages.items()}
    out["stages_of"] = (f"roofline pass: camera stream 0 alone, {steps} steps of {B} frames "
                        f"after the timed region")
    out["extract_vs_match"] = phase_split(stages, steps, B)
    return out


EXTRACT_STAGES = ("k_pyramid", "k_blur", "k_fast_cells", "k_octree", "k_describe", "k_cvfast", "k_cvselect", "k_cvdescribe")


def phase_split(stages, steps, B):
    """SURVEY §8d asks for "extract" and "match" rates beside the combined one: the stage times
    of the roofline pass (one camera stream alone) summed per phase, as ms per batch of B frames
    and the frames/s one stream would reach on that phase alone (the timed region overlaps
    several streams, so these do not add up to `value`)."""
    ex = sum(v[0] for k, v in stages.items() if k in EXTRACT_STAGES) / steps
    ma = sum(v[0] for k, v in stages.items() if k not in EXTRACT_STAGES) / steps
    fps = lambda ms: round(B / (ms / 1e3), 1) if ms > 0 else None  # noqa: E731
    return {"extract_ms_per_batch": round(ex, 4), "match_ms_per_batch": round(ma, 4),
            "extract_frames_per_s_one_stream": fps(ex), "match_frames_per_s_one_stream": fps(ma),
            "combined_frames_per_s_one_stream": fps(ex + ma),
            "match_stages": sorted(k for k in stages if k not in EXTRACT_STAGES)}


# ---------------------------------------------------------------------------- CPU baseline
def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.gnu_get_libc_version.restype = ctypes.c_char_p
        glibc = libc.gnu_get_libc_version().decode()
    except (OSError, AttributeError):
        glibc = None
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    # the process's CPU share: on the GPU box the affinity mask shows the whole machine while
    # OMP_NUM_THREADS (16 per GPU) states the share a job may use
    share = int(os.environ.get("OMP_NUM_THREADS") or 0)
    if share > 0:
        cores = min(cores, share)
    return {"cpu_model": model or platform.processor() or platform.machine(),
            "cores_available": cores, "glibc": glibc,
            "glibc_note": "descriptor parity is defined against this glibc's sincosf "
                          "(the reference calls sincosf; SURVEY App. C.2)"}


class CpuUnit:
    """The CPU oracle's unit of work (orb_oracle.cc restating ORBextractor/ORBmatcher, DBoW2
    restatement): extract (x2 + ComputeStereoMatches for stereo) + ComputeBoW + SearchByBoW +
    SearchForTriangulation against the previous frame of the same stream."""

    def __init__(self, cfg, n_images=16, stream=0):
        from oracle import oracle as O
        from ar_orbslam2_amd import synth
        from ar_orbslam2_amd.pipeline import TUM1_K, fundamental_from_pose
        from ar_orbslam2_amd.vocabulary import complete_tree
        self.O = O
        self.cfg = cfg
        w, h, nf = cfg["w"], cfg["h"], cfg["nfeatures"]
        self.p = O.params(nf)
        self.t = O.tables(self.p, w, h)
        ndesc = sum(10 ** l for l in range(7))
        self.voc = O.Vocabulary.from_nodes(10, 6, 0, 0, *complete_tree(
            10, 6, np.random.default_rng(42).integers(0, 256, (ndesc, 32), dtype=np.uint8)))
        self.F = fundamental_from_pose()
        self.ex, self.ey = O.epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
        self.stereo = cfg.get("stereo")
        if self.stereo:
            from ar_orbslam2_amd.stereo import stereo_params
            self.mb, self.mbf = stereo_params(*self.stereo)
            self.imgs = [synth.stereo_pair(w, h, i, stream) for i in range(n_images)]
        else:
            base = synth.canvas(w, h, stream)
            self.imgs = [synth.frame(w, h, i, stream, base) for i in range(n_images)]
        self.prev = None
        self.n = 0

    def step(self):
        O, t = self.O, self.t
        img = self.imgs[self.n % len(self.imgs)]
        u_right = None
        if self.stereo:
            kps, desc, pl, _ = O.extract(img[0], self.p, want_pyramid=True)
            kr, dr, pr, _ = O.extract(img[1], self.p, want_pyramid=True)
            u_right = O.stereo_matches(kps, desc, kr, dr, pl, pr, t["scale"], t["inv_scale"],
                                       self.mb, self.mbf)[0]
        else:
            kps, desc = O.extract(img, self.p)
        b = self.voc.transform(desc, 4)  # Frame::ComputeBoW: BowVector + FeatureVector
        r = np.random.default_rng(self.n)
        cur = dict(desc=desc, angle=kps["angle"], keys=kps,
                   fv=(b["fv_ids"], b["fv_off"], b["fv_feats"]),
                   valid=(r.random(len(kps)) < 0.6).astype(np.uint8),
                   has_mp=(r.random(len(kps)) < 0.4).astype(np.uint8), u_right=u_right,
                   scale_factors=t["scale"], level_sigma2=t["sigma2"])
        if self.prev is not None:
            O.search_by_bow_kf_f(self.prev, dict(cur, valid=None), 0.7, True)
            O.search_for_triangulation(self.prev, cur, self.F, self.ex, self.ey, False, 0.6, False)
        self.prev = cur
        self.n += 1


def _cpu_worker(unit, seconds, start_evt, q):
    for _ in range(3):  # warm-up
        unit.step()
    start_evt.wait()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        unit.step()
        n += 1
    q.put((n, time.perf_counter() - t0))


def cpu_baseline(cfg, seconds, mp_seconds, warmup=20, min_frames=200, max_seconds=40.0):
    """SURVEY §8d CPU baseline, measured on this host before any GPU work of this process:
    * one thread: `warmup` untimed frames, then frames timed one by one (steady clock) until
      >= min_frames and >= `seconds` (or `max_seconds`); median and mean ms per frame, as
      mono_tum.cc:113-121 reports tracking times;
    * every available core (sched_getaffinity): one forked process per core, each its own
      camera stream, aggregate frames/s over `mp_seconds` — the `value`."""
    import multiprocessing as mp
    info = host_info()
    unit = CpuUnit(cfg)
    for _ in range(warmup):
        unit.step()
    times = []
    t0 = time.perf_counter()
    while True:
        a = time.perf_counter()
        unit.step()
        times.append(time.perf_counter() - a)
        el = time.perf_counter() - t0
        if (len(times) >= min_frames and el >= seconds) or el >= max_seconds:
            break
    times_ms = np.array(times) * 1e3
    single = {"frames_per_s": round(len(times) / el, 3), "median_ms": round(float(np.median(times_ms)), 3),
              "mean_ms": round(float(times_ms.mean()), 3), "timed_frames": len(times),
              "warmup_frames": warmup}
    P = info["cores_available"] or 1
    ctx = mp.get_context("fork")  # no GPU work has happened in this process yet
    start, q = ctx.Event(), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(CpuUnit(cfg, 8, stream=1 + i), mp_seconds, start, q))
             for i in range(P)]
    for p in procs:
        p.start()
    time.sleep(0.5)
    start.set()
    res = [q.get(timeout=mp_seconds * 4 + 120) for _ in procs]
    for p in procs:
        p.join()
    agg = sum(n for n, _ in res) / max(e for _, e in res)
    stereo = cfg.get("stereo")
    w, h = cfg["w"], cfg["h"]
    unit_desc = (f"extract{' x2 + ComputeStereoMatches' if stereo else ''} + ComputeBoW + "
                 f"SearchByBoW + SearchForTriangulation per frame")
    return dict(value=round(agg, 3), unit="frames/s", cores=P, kind="port",
                sample=f"{w}x{h} synthetic {'stereo ' if stereo else ''}frames, CPU oracle "
                       f"(oracle/*.cc, g++ -O3 -march=x86-64-v4 -mtune=znver3 -ffp-contract=off): {P} forked "
                       f"processes x 1 thread, one camera stream each, {mp_seconds:.0f} s after 3 "
                       f"warm-up frames ({sum(n for n, _ in res)} frames); {unit_desc}",
                single_thread=single, **info)


class MarkerUnit:
    """One marker-path frame of the CPU oracle (cvorb_oracle.cc): cv::ORB of the frame,
    BruteForceMatcher match against the target's descriptors, Marker::Match's good filter.
    The target is the one run_marker builds (synth.frame(w, h, 5, 0)); its oracle descriptors
    are the GPU's (tests/test_cvorb_gpu.py)."""

    def __init__(self, cfg, n_images=32, stream=0):
        from oracle import oracle as O
        from ar_orbslam2_amd import synth
        self.O = O
        w, h = cfg["w"], cfg["h"]
        self.p = O.cvorb_params(cfg["nfeatures"])
        self.target_desc = O.cvorb_detect(synth.frame(w, h, 5, 0), self.p)[1]
        base = synth.canvas(w, h, stream)
        self.imgs = [synth.frame(w, h, i, stream, base) for i in range(n_images)]
        self.n = 0

    def step(self):
        O = self.O
        desc = O.cvorb_detect(self.imgs[self.n % len(self.imgs)], self.p)[1]
        O.good_matches(O.bf_match(self.target_desc, desc))
        self.n += 1


def cpu_baseline_marker(cfg, seconds, mp_seconds, warmup=5, min_frames=100, max_seconds=40.0):
    """The marker path's CPU baseline, before any GPU work of this process, as cpu_baseline:
    one thread timed frame by frame (median / mean ms), and `value` = every available core, one
    forked process per core on its own camera stream."""
    import multiprocessing as mp
    info = host_info()
    unit = MarkerUnit(cfg)
    for _ in range(warmup):
        unit.step()
    times = []
    t0 = time.perf_counter()
    while True:
        a = time.perf_counter()
        unit.step()
        times.append(time.perf_counter() - a)
        el = time.perf_counter() - t0
        if (len(times) >= min_frames and el >= seconds) or el >= max_seconds:
            break
    ms = np.array(times) * 1e3
    single = {"frames_per_s": round(len(times) / el, 3), "median_ms": round(float(np.median(ms)), 3),
              "mean_ms": round(float(ms.mean()), 3), "timed_frames": len(times),
              "warmup_frames": warmup}
    P = info["cores_available"] or 1
    ctx = mp.get_context("fork")  # no GPU work has happened in this process yet
    start, q = ctx.Event(), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(MarkerUnit(cfg, 8, stream=1 + i), mp_seconds, start, q))
             for i in range(P)]
    for p in procs:
        p.start()
    time.sleep(0.5)
    start.set()
    res = [q.get(timeout=mp_seconds * 4 + 120) for _ in procs]
    for p in procs:
        p.join()
    agg = sum(n for n, _ in res) / max(e for _, e in res)
    w, h = cfg["w"], cfg["h"]
    return dict(value=round(agg, 3), unit="frames/s", cores=P, kind="port",
                sample=f"{w}x{h} synthetic frames, CPU oracle (oracle/cvorb_oracle.cc, g++ -O3 "
                       f"-march=x86-64-v4 -mtune=znver3 -ffp-contract=off): {P} forked processes x 1 thread, one "
                       f"camera stream each, {mp_seconds:.0f} s after 3 warm-up frames "
                       f"({sum(n for n, _ in res)} frames); cv::ORB + BruteForceMatcher vs "
                       f"{len(unit.target_desc)} target descriptors + good filter per frame",
                single_thread=single, **info)


def cvorb_level_sizes(params, w, h):
    """cv::ORB 2.4 pyramid sizes (orb.cpp operator(): scale = (float)pow(scaleFactor, level),
    size = cvRound(cols * (1 / scale))) — host arithmetic for the byte model, computed here so
    that the product leg of bench.py never calls into oracle/."""
    sf = float(params.scale_factor)
    out = []
    for lvl in range(params.nlevels):
        inv = np.float32(1) / np.float32(sf ** (lvl - params.first_level))
        out.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return out


def marker_bytes(levels, n_kp, n_img, n_target):
    """Algorithmic bytes per launch of the marker-path kernels (same byte model as §8d; the
    matcher reads both descriptor sets once per frame)."""
    P = [w * h for w, h in levels]
    per_resize = [(P[l - 1] + P[l]) * n_img for l in range(1, len(P))]
    return {"k_pyramid": 2 * P[0] * n_img + sum(per_resize),
            "k_cvfast": sum(P) * n_img, "k_blur": 2 * sum(P) * n_img,
            "k_cvselect": sum(P) * n_img / 8 + 8 * n_kp, "k_cvdescribe": 60 * n_kp,
            "k_bfmatch": 32 * (n_kp + n_target * n_img) + 8 * n_target * n_img,
            "k_good": 24 * n_target * n_img}


# ---------------------------------------------------------------------------- distribution
def aggregate_elapsed(elapsed, world):
    """Max over ranks: the job is as fast as its slowest GPU (RCCL/gloo all_reduce MAX)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def streams_of_rank(rank, world, streams_per_gpu=1, streams_total=None):
    """Global camera-stream ids processed by `rank` (stream s -> GPU s mod G, no
    exchange).  Weak scaling: G x streams_per_gpu streams in the job; strong scaling: a fixed
    `streams_total`, each rank taking the ids congruent to it mod G."""
    total = streams_total if streams_total else world * max(1, streams_per_gpu)
    return [s for s in range(total) if s % world == rank]


def stream_of_rank(rank):
    """First camera stream of a rank (one stream per rank)."""
    return streams_of_rank(rank, rank + 1)[0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n, argv):
    """`--gpus N` without a launcher: start N rank processes (RANK = LOCAL_RANK = r, one GPU
    each) and wait for them.  Called before this process touches the GPU; rank 0 prints the
    JSON line.  Returns the worst exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


def init_dist(rank, world, local, backend):
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def gather_streams(streams, world):
    if world <= 1:
        return [streams]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, streams)
    return out


def run_dry(args, cfg, rank, world, streams):
    """--dry-run: the launcher, stream sharding and max-over-ranks aggregation without device
    work (gloo), for the CPU tests of the N>1 path."""
    dist = init_dist(rank, world, rank, "gloo")
    all_streams = gather_streams(streams, world)
    B = args.batch
    frames = sum(len(s) for s in all_streams) * B * args.steps
    elapsed = aggregate_elapsed(0.01 * (1 + rank), world)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(frames / elapsed, 2), "unit": "frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if args.streams_total else "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic", "dry_run": True,
            "config": {"workload": cfg["workload"], "streams_per_rank": all_streams,
                       "frames_per_batch": B}}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


# ---------------------------------------------------------------------------- GPU legs
def upload_pass(pipes, pools_host, B, steps, torch):
    """PCIe-included rate: every step's frames start in pinned host memory and are copied to
    HBM on one copy stream (double-buffered per camera stream, overlapped with the previous
    batch's graph on the pipeline stream; one copy stream keeps the job within the box's 4
    hardware queues: S pipeline streams + 1).  Also times the bare H2D of the same bytes."""
    S = len(pipes)
    nbytes = pools_host[0][0].numel()
    dbuf = [[torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(2)]
            for _ in range(S)]
    cs_all = torch.cuda.Stream()
    cstreams = [cs_all] * S
    pstreams = [torch.cuda.ExternalStream(p.stream()) for p in pipes]
    up = [[torch.cuda.Event() for _ in range(2)] for _ in range(S)]
    done = [[torch.cuda.Event() for _ in range(2)] for _ in range(S)]

    def step(i):
        k = i % 2
        for si, p in enumerate(pipes):
            cs = cstreams[si]
            cs.wait_event(done[si][k])  # the graph that last read dbuf[k] has finished
            with torch.cuda.stream(cs):
                dbuf[si][k].copy_(pools_host[si][i % len(pools_host[si])], non_blocking=True)
                up[si][k].record(cs)
            pstreams[si].wait_event(up[si][k])
            p.run(dbuf[si][k].data_ptr(), B)
            done[si][k].record(pstreams[si])

    for i in range(2):
        step(i)
    for p in pipes:
        p.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    for p in pipes:
        p.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # bare H2D of the same bytes (copy streams only)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(steps):
        for si in range(S):
            with torch.cuda.stream(cstreams[si]):
                dbuf[si][i % 2].copy_(pools_host[si][i % len(pools_host[si])], non_blocking=True)
    torch.cuda.synchronize()
    el_copy = time.perf_counter() - t1
    frames = S * B * steps
    gbs = S * nbytes * steps / el / 1e9
    copy_gbs = S * nbytes * steps / el_copy / 1e9
    return {"value": round(frames / el, 2), "unit": "frames/s",
            "h2d_GBs": round(gbs, 2), "h2d_copy_only_GBs": round(copy_gbs, 2),
            "pcie_spec_GBs": PCIE_GEN5_X16_GBS,
            "frac_of_pcie_spec": round(gbs / PCIE_GEN5_X16_GBS, 4),
            "frac_of_copy_only": round(gbs / copy_gbs, 4),
            "frames_ceiling_at_spec": round(PCIE_GEN5_X16_GBS * 1e9 / (nbytes / B), 1),
            "note": "frames start in pinned host memory; H2D on one copy stream, "
                    "double-buffered per camera stream, overlapped with the previous batch's graph"}


def run_marker(args, cfg, rank, world, local, streams, dist):
    import torch
    from ar_orbslam2_amd import synth
    from ar_orbslam2_amd.marker import ORB, MarkerBatch, cvorb_params
    w, h, nf, B = cfg["w"], cfg["h"], cfg["nfeatures"], args.batch
    S = len(streams)
    # the target's descriptors come from the product cv::ORB (Marker::setTargetImage)
    target = synth.frame(w, h, 5, 0)
    orb = ORB(nf, size=(w, h), device=local)
    _, target_desc = orb(target)
    orb.close()
    pipes, pools = [], []
    for stream_id in streams:
        mb = MarkerBatch(w, h, B, nf, device=local)
        mb.set_target(target_desc)
        base = synth.canvas(w, h, stream=stream_id)
        pool = []
        for pi in range(args.pool):
            fr = np.stack([synth.frame(w, h, pi * B + i, stream_id, base) for i in range(B)])
            pool.append(torch.from_numpy(fr).cuda())
        pipes.append(mb)
        pools.append(pool)
    torch.cuda.synchronize()

    def barrier():
        if dist:
            dist.barrier()

    for i in range(args.warmup):
        for p, pool in zip(pipes, pools):
            p.run(pool[i % len(pool)].data_ptr(), B)
    for p in pipes:
        p.sync()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        for p, pool in zip(pipes, pools):
            p.run(pool[i % len(pool)].data_ptr(), B)
    for p in pipes:
        p.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    stages, kernels = {}, {}
    pipe = pipes[0]
    if not args.no_profile:
        pipe.profile(True)
        for i in range(args.roofline_steps):
            pipe.run(pools[0][i % len(pools[0])].data_ptr(), B)
        pipe.sync()
        stages = pipe.profile_read()
        kernels = pipe.profile_kernels()
        pipe.profile(False)
    kp_counts, good_counts = pipe.results(B)
    if (kp_counts < 0).any():
        raise RuntimeError("a frame overflowed the per-level keypoint capacity")
    elapsed = aggregate_elapsed(elapsed, world)
    n_streams = sum(len(x) for x in gather_streams(list(streams), world))
    value = n_streams * B * args.steps / elapsed
    levels = cvorb_level_sizes(cvorb_params(nf), w, h)
    n_kp = int(kp_counts.sum())
    alg = marker_bytes(levels, n_kp, B, len(target_desc))
    roofline = roofline_of(stages, alg, args.pmc_dir, args.roofline_steps, B, kernels)
    out = {
        "metric": MARKER_METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if args.streams_total else "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "frames_per_step_per_gpu": B * S,
                   "camera_streams_per_gpu": S, "camera_streams_total": n_streams,
                   "frames_per_batch": B, "image": f"{w}x{h}",
                   "nfeatures": nf, "target_descriptors": len(target_desc),
                   "parallelism": f"{world} GPU(s), camera stream s on GPU s mod {world}, "
                                  f"no collective",
                   "keypoints_per_frame": round(n_kp / B, 1),
                   "good_matches_per_frame": round(float(good_counts.mean()), 1),
                   "hamming_pairs_per_frame": round(n_kp / B * len(target_desc)),
                   "timing": "hipGraph replay of the extraction + 2 matcher launches per batch"},
        "roofline": roofline,
    }
    out["config"]["library"] = library_info()
    return out, target_desc


def _gen_pool(fn, n, threads=16):
    """n synthetic frames fn(i) in order; numpy's generators and ufuncs release the GIL, so a
    thread pool spreads the host-side generation over the job's CPU share."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max(1, min(threads, n))) as ex:
        return list(ex.map(fn, range(n)))


def make_frame_pipes(args, cfg, streams, local):
    """The timed topology of run_frames: one FramePipeline (own HIP stream, captured hipGraphs)
    per camera stream with SURVEY §8d's seeded masks and matcher settings, and `args.pool`
    distinct batches of B frames of that stream resident in HBM.  Returns (pipes, pools,
    pools_host): pools[s][k] is a device tensor, pools_host[s] the pinned copies of the first
    two batches for the PCIe leg (None without --upload).  Each pipe carries `masks` (valid,
    has_mp) and `epipole`.  tests/test_pipeline_gpu.py builds the same topology through this
    function and checks its outputs against the oracle."""
    import torch
    from ar_orbslam2_amd import Vocabulary, epipole, synth
    from ar_orbslam2_amd.pipeline import TUM1_K, FramePipeline, fundamental_from_pose

    w, h, nf, B = cfg["w"], cfg["h"], cfg["nfeatures"], args.batch
    voc = Vocabulary.synthetic(device=local)
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    pipes, pools, pools_host = [], [], []
    stereo = None
    if cfg.get("stereo"):
        from ar_orbslam2_amd.stereo import stereo_params
        stereo = stereo_params(*cfg["stereo"])
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
    for stream_id in streams:
        pipe = FramePipeline(w, h, B, voc, nf, device=local, stereo=stereo)
        pipe.masks = pipe.seeded_masks(range(B))
        pipe.epipole = (ex, ey)
        pipe.set_matching(fundamental_from_pose(), (ex, ey), bow_ratio=0.7, bow_check_ori=True,
                          tri_ratio=0.6, tri_check_ori=False)
        # synthetic frames of this camera stream, resident in HBM before timing
        host = []
        if stereo:
            pairs = _gen_pool(lambda t: synth.stereo_pair(w, h, t, stream_id), min(B, 32), threads)
            for pi in range(args.pool):  # interleaved (left, right) images
                host.append(np.stack([im for i in range(B) for im in pairs[(pi * 7 + i) % len(pairs)]]))
        else:
            base = synth.canvas(w, h, stream=stream_id)
            allf = _gen_pool(lambda i: synth.frame(w, h, i, stream_id, base), args.pool * B, threads)
            for pi in range(args.pool):
                host.append(np.stack(allf[pi * B:(pi + 1) * B]))
            del allf
        pools.append([torch.from_numpy(fr).cuda() for fr in host])
        pools_host.append([torch.from_numpy(fr).reshape(-1).pin_memory() for fr in host[:2]]
                          if args.upload else None)
        pipes.append(pipe)
    torch.cuda.synchronize()
    return pipes, pools, pools_host


def _d2h(ptr, nbytes):
    """Device bytes at `ptr` (a pipeline output) to a host u8 array (hipMemcpy D2H)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.zeros(nbytes, np.uint8)
    rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr),
                       ctypes.c_size_t(nbytes), 2)
    if rc != 0:
        raise RuntimeError(f"hipMemcpy D2H failed ({rc})")
    return out


def dump_verify_frames(out_dir, rank, stream_id, pipe, batch, B, stereo):
    """--verify-frames: this rank's first camera stream, the batch its last timed step ran —
    frames {0, B-1} with their keyframes {B-1, B-2} (frame f is matched against (f - 1) mod B):
    input images, keypoints, descriptors, (stereo) mvuRight / mvDepth, SearchByBoW matches,
    SearchForTriangulation pairs and the masks, to out_dir/rank{rank}.npz.  Every rank's outputs
    can then be checked against the oracle (tests/test_distributed_gpu.py), not only rank 0's
    counts."""
    from ar_orbslam2_amd import KEYPOINT_DTYPE
    pipe.sync()
    cap = pipe.kp_cap
    ni = 2 * B if stereo else B
    counts, bow, tri, err = pipe.results(B)
    out = pipe.device_outputs()
    ids = [B - 2, B - 1, 0]
    imgs = batch.cpu().numpy()
    img_rows = [j for f in ids for j in ((2 * f, 2 * f + 1) if stereo else (f,))]
    kps = _d2h(out["kps"], ni * cap * 28).view(KEYPOINT_DTYPE).reshape(ni, cap)
    desc = _d2h(out["desc"], ni * cap * 32).reshape(ni, cap, 32)
    match = _d2h(out["bow_match"], B * cap * 4).view(np.int32).reshape(B, cap)
    pairs = _d2h(out["tri_pairs"], B * cap * 8).view(np.int32).reshape(B, cap, 2)
    valid, has_mp = pipe.masks
    d = dict(rank=rank, stream=stream_id, batch=B, stereo=int(stereo), frame_ids=np.array(ids),
             err=err, counts=counts[ids], images=imgs[img_rows], kps=kps[img_rows],
             desc=desc[img_rows], bow=bow[[0, B - 1]], match=match[[0, B - 1]],
             tri=tri[[0, B - 1]], pairs=pairs[[0, B - 1]], valid=valid[ids], has_mp=has_mp[ids],
             epipole=np.array(pipe.epipole, np.float32))
    if stereo:
        so = pipe.stereo_outputs()
        d["uright"] = _d2h(so["uright"], B * cap * 4).view(np.float32).reshape(B, cap)[ids]
        d["depth"] = _d2h(so["depth"], B * cap * 4).view(np.float32).reshape(B, cap)[ids]
    os.makedirs(out_dir, exist_ok=True)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **d)


def replay_step(pipes, pools, B, i):
    """One step of the timed region: every camera stream enqueues batch i mod pool (its
    captured hipGraph for that input, replayed asynchronously on the pipeline's stream)."""
    for p, pool in zip(pipes, pools):
        p.run(pool[i % len(pool)].data_ptr(), B)


def run_frames(args, cfg, rank, world, local, streams, dist):
    import torch
    from ar_orbslam2_amd import ORBextractor

    w, h, nf, B = cfg["w"], cfg["h"], cfg["nfeatures"], args.batch
    stereo = cfg.get("stereo")
    S = len(streams)
    pipes, pools, pools_host = make_frame_pipes(args, cfg, streams, local)
    pipe = pipes[0]

    def barrier():
        if dist:
            dist.barrier()

    # setup: one run per resident batch captures every (input, batch) hipGraph before the
    # warm-up, so no capture lands in the timed region when the pool is larger than W
    for i in range(len(pools[0])):
        replay_step(pipes, pools, B, i)
    for i in range(args.warmup):
        replay_step(pipes, pools, B, i)
    for p in pipes:
        p.sync()
        if p.results(B)[3]:
            raise RuntimeError(f"frame pipeline reported device error {p.results(B)[3]}")

    # timed region: every camera stream replays its captured hipGraph, no per-kernel events
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        replay_step(pipes, pools, B, i)
    for p in pipes:
        p.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    for si, p in enumerate(pipes):
        if p.results(B)[3]:
            raise RuntimeError(f"camera stream {streams[si]}: device error {p.results(B)[3]}")
    if args.verify_frames:
        dump_verify_frames(args.verify_frames, rank, streams[0], pipes[0],
                           pools[0][(args.steps - 1) % len(pools[0])], B, bool(stereo))
    # roofline pass (after timing): stream 0 alone with HIP events around every kernel on the
    # stream it launches on, so a kernel's event interval is its own duration (as rocprofv3
    # reports it) rather than a share of the concurrent streams
    stages, kernels = {}, {}
    if not args.no_profile:
        pipe.profile(True)
        for i in range(args.roofline_steps):
            pipe.run(pools[0][i % len(pools[0])].data_ptr(), B)
        pipe.sync()
        stages = pipe.profile_read()
        kernels = pipe.profile_kernels()
        pipe.profile(False)
    kp_counts, bow, tri, err = pipe.results(B)
    if err:
        raise RuntimeError(f"frame pipeline reported device error {err}")
    upload = None
    if args.upload:
        del pools  # the device-resident pools are not needed any more
        upload = upload_pass(pipes, pools_host, B, args.steps, torch)

    elapsed = aggregate_elapsed(elapsed, world)
    # every rank's camera streams (stream s on rank s mod G); the job's frames are
    # the sum over the ranks' streams
    all_streams = gather_streams(list(streams), world)
    n_streams = sum(len(x) for x in all_streams)
    frames_total = n_streams * B * args.steps
    value = frames_total / elapsed
    ex_tables = ORBextractor(nf, device=local)
    levels = level_sizes(w, h, ex_tables.GetInverseScaleFactors())
    n_kp = int(kp_counts.sum())
    # stereo: both images of a frame are extracted (right keypoint count ~ left)
    alg = algorithmic_bytes(levels, 2 * n_kp if stereo else n_kp, 2 * B if stereo else B)
    roofline = roofline_of(stages, alg, args.pmc_dir, args.roofline_steps, B, kernels)
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if args.streams_total else "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "frames_per_step_per_gpu": B * S,
                   "camera_streams_per_gpu": S, "camera_streams_total": n_streams,
                   "frames_per_batch": B,
                   "image": f"{w}x{h}", "images_per_frame": 2 if stereo else 1,
                   "nfeatures": nf, "nlevels": 8, "scale_factor": 1.2,
                   "parallelism": f"{world} GPU(s), camera stream s on GPU s mod {world}, "
                                  f"no collective",
                   "streams_per_rank": all_streams, "frames_total": frames_total,
                   "dist_backend": args.dist_backend if world > 1 else None,
                   "same_device": bool(args.same_device),
                   "keypoints_per_frame": round(n_kp / B, 1),
                   "bow_matches_per_frame": round(float(bow.mean()), 1),
                   "triangulation_matches_per_frame": round(float(tri.mean()), 1),
                   "timing": "hipGraph replay (every pool batch's graph captured in setup, "
                             "before the warm-up); per-kernel HIP events only in the roofline pass"},
        "roofline": roofline,
    }
    out["config"]["library"] = library_info()
    if upload:
        out["pcie_upload_included"] = upload
    return out


class _nullctx:
    def __init__(self, v):
        self.v = v

    def __enter__(self):
        return self.v

    def __exit__(self, *a):
        return False


def run_dropin(args, cfg, rank, world, local):
    """--dropin: the per-frame path ORB-SLAM2 calls (Frame.cc:252-258 -> ORBextractor::operator(),
    Frame::ComputeBoW, ORBmatcher::SearchByBoW / SearchForTriangulation one frame or keyframe
    pair per call, Tracking.cc:1132-1136, LocalMapping.cc:238-241), driven by the C++ program
    tools/orbx_dropin.cpp over liborbx.so from pageable host images (cv::Mat), K host threads
    each with its own extractor (one per camera, like the reference's per-camera ORBextractor).
    Runs as a child process; this process never touches the GPU."""
    import tempfile
    from ar_orbslam2_amd import synth
    from ar_orbslam2_amd.vocabulary import complete_tree
    from ar_orbslam2_amd import _ffi  # the library directory (an experiment build's with ORBX_LIB_DIR)
    exe = os.path.join(os.path.dirname(_ffi.LIB_PATH), "orbx_dropin")
    if not os.path.exists(exe):
        raise FileNotFoundError(f"{exe} missing: build with __graft_entry__.build()")
    w, h, nf = cfg["w"], cfg["h"], cfg["nfeatures"]
    n_img = 32
    keep = args.dropin_dir
    if keep:
        os.makedirs(keep, exist_ok=True)
    with (tempfile.TemporaryDirectory() if not keep else _nullctx(keep)) as td:
        fr = np.stack([synth.frame(w, h, i, s) for s in range(args.threads) for i in range(n_img)])
        fr.tofile(os.path.join(td, "frames.u8"))
        ndesc = sum(10 ** l for l in range(7))
        parent, is_leaf, desc, weight = complete_tree(
            10, 6, np.random.default_rng(42).integers(0, 256, (ndesc, 32), dtype=np.uint8))
        parent.astype(np.int32).tofile(os.path.join(td, "voc_parent.i32"))
        is_leaf.astype(np.uint8).tofile(os.path.join(td, "voc_leaf.u8"))
        desc.astype(np.uint8).tofile(os.path.join(td, "voc_desc.u8"))
        weight.astype(np.float64).tofile(os.path.join(td, "voc_weight.f64"))
        cmd = [exe, td, str(w), str(h), str(nf), str(n_img), str(args.threads),
               str(args.warmup_frames), str(args.dropin_frames), str(local), args.dropin_mode]
        if keep:  # inputs kept for a profiler run of the driver itself
            with open(os.path.join(keep, "cmd.txt"), "w") as f:
                f.write(" ".join(cmd[1:]) + "\n")
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if res.returncode != 0:
        raise RuntimeError(f"orbx_dropin failed ({res.returncode}): {res.stderr[-2000:]}")
    d = json.loads(res.stdout.strip().splitlines()[-1])
    return {
        "metric": METRIC + " (drop-in per-frame path, host images)", "value": d["fps"],
        "unit": "frames/s", "n_gpus": 1, "steps": d["frames"], "warmup": args.warmup_frames,
        "ms_per_step": d["mean_ms"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"] + (", drop-in C ABI one frame per call"
                                                  if args.dropin_mode == "capi" else
                                                  ", drop-in through the reference-side shims' "
                                                  "per-call marshalling, one frame per call"),
                   "host_threads": args.threads, "image": f"{w}x{h}", "nfeatures": nf,
                   "dropin_mode": args.dropin_mode, "library": library_info()},
        "dropin": d,
    }


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per step per camera stream (default: the config's, else 256)")
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--pool", type=int, default=4, help="distinct resident batches cycled")
    ap.add_argument("--streams", type=int, default=3,
                    help="weak scaling: independent camera-stream pipelines per GPU, one HIP "
                         "stream each (concurrent streams fill the CUs the serial stages leave idle)")
    ap.add_argument("--streams-total", type=int, default=None,
                    help="strong scaling: the job's camera-stream count, fixed over the GPUs "
                         "(stream s on GPU s mod G); e.g. C5's 8 streams")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for the barrier and the max-over-ranks time "
                         "(nccl = RCCL; no data-path collective either way)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank uses device 0: rehearses the N>1 path on a one-GPU box "
                         "(with --dist-backend gloo; RCCL refuses two ranks on one GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + sharding + aggregation only, no device work (gloo)")
    ap.add_argument("--upload", dest="upload", action="store_true", default=True,
                    help="also measure the rate with frames uploaded from pinned host memory")
    ap.add_argument("--no-upload", dest="upload", action="store_false")
    ap.add_argument("--dropin", action="store_true",
                    help="measure the drop-in per-frame path (host images, one frame per call)")
    ap.add_argument("--dropin-mode", default="capi", choices=["capi", "shim"],
                    help="--dropin: call the C ABI directly (capi) or replay the reference-side "
                         "shims' per-call marshalling around it (shim: std::map BoW / "
                         "FeatureVector, MapPoint masks, per-call buffers; include/compat)")
    ap.add_argument("--threads", type=int, default=4, help="--dropin host threads (cameras)")
    ap.add_argument("--dropin-frames", type=int, default=500, help="--dropin frames per thread")
    ap.add_argument("--warmup-frames", type=int, default=20, help="--dropin warm-up per thread")
    ap.add_argument("--dropin-dir", default=None,
                    help="--dropin: keep the driver's inputs (and its arguments in cmd.txt) here")
    ap.add_argument("--verify-frames", default=None, metavar="DIR",
                    help="after the timed region, every rank dumps frames {0, B-1} of its first "
                         "camera stream (inputs, keypoints, descriptors, matches) to "
                         "DIR/rank<r>.npz for an oracle check of that rank's outputs")
    ap.add_argument("--pmc-dir", default=None,
                    help="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ CSVs of this bench command, "
                         "used for roofline.traffic and the VALU-issue floor")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="single-thread CPU baseline: at least this long and 200 frames")
    ap.add_argument("--cpu-mp-seconds", type=float, default=6.0,
                    help="all-cores CPU baseline window")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the per-kernel roofline pass after the timed region")
    ap.add_argument("--roofline-steps", type=int, default=5,
                    help="steps of the single-stream roofline pass (per-kernel HIP events)")
    args = ap.parse_args(argv)
    if args.batch is None:
        args.batch = CONFIGS[args.config].get("batch", 256)
    if args.pmc_dir is None:  # this round's committed PMC passes of the config's default command
        # (never another config's; passes of another library build or without the timed kernel
        # instances give null counter fields with the reason, pmc_binding)
        args.pmc_dir = os.path.join(ROOT, "profiles",
                                    f"{PMC_ROUND}_pmc" if args.config == "C2" else
                                    f"{PMC_ROUND}_pmc_" + args.config.lower())
    return args


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.dropin:
        sys.exit(spawn_ranks(args.gpus, argv))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", str(rank)))
    if args.same_device and args.dist_backend == "nccl" and world > 1:
        raise SystemExit("--same-device needs --dist-backend gloo (RCCL refuses two ranks on one GPU)")
    if args.streams_total is not None and args.streams_total < world:
        raise SystemExit(f"--streams-total {args.streams_total} < {world} GPUs")
    streams = streams_of_rank(rank, world, args.streams, args.streams_total)
    cfg = CONFIGS[args.config]
    if args.dry_run:
        run_dry(args, cfg, rank, world, streams)
        return
    if args.dropin:
        out = run_dropin(args, cfg, rank, world, local)
        print(json.dumps(out), flush=True)
        return
    # the CPU baseline runs first, before this process touches the GPU (its all-cores leg
    # forks one process per core) and without the GPU leg's host threads competing
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = (cpu_baseline_marker if cfg.get("marker") else cpu_baseline)(
            cfg, args.cpu_seconds, args.cpu_mp_seconds)
    import torch
    torch.cuda.set_device(local)
    dist = init_dist(rank, world, local, args.dist_backend)
    if cfg.get("marker"):
        out, _ = run_marker(args, cfg, rank, world, local, streams, dist)
    else:
        out = run_frames(args, cfg, rank, world, local, streams, dist)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
