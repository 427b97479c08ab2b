#!/usr/bin/env python3
"""Benchmark: frames/s of ORB extract + match (BASELINE.json metric) on MI355X.

One step = one batch of `--batch` synthetic 640x480 frames (BASELINE.json configs[1], TUM
fr1/xyz mono geometry, 1000 features) already resident in HBM, pushed through the whole
device pipeline: ORBextractor (pyramid, FAST cells, octree, orientation, rBRIEF),
Frame::ComputeBoW (full DBoW2 descent of the seeded k=10, L=6 vocabulary: word ids, BowVector,
FeatureVector), SearchByBoW(prev-as-KF, cur) and SearchForTriangulation(prev-as-KF, cur-as-KF)
(SURVEY §8d unit of work).  Multi-GPU: one process per GPU, each rank processes its
own camera stream (weak scaling, no data-path collective; RCCL only carries the barrier and
the max-over-ranks time).

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (HIP events on the
pipeline stream over the timed region) and the CPU oracle baseline (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match, 640×480 1000-feat; bit-exact descriptors"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CONFIGS = {
    "C2": dict(w=640, h=480, nfeatures=1000,
               workload="TUM fr1/xyz mono 640x480, 1000 features, 1xMI355X HIP extract+match"),
    "C3": dict(w=752, h=480, nfeatures=1200, stereo=(47.90639384423901, 435.2046959714599),
               workload="EuRoC MH01 stereo geometry 2x752x480, 1200 features, stereo matching"),
    "C4": dict(w=1241, h=376, nfeatures=2000, stereo=(386.1448, 718.856),
               workload="KITTI 00 stereo geometry 2x1241x376, 2000 features, stereo matching"),
    "C5": dict(w=1920, h=1080, nfeatures=4000, workload="synthetic 1920x1080, 4000 features"),
    # the AR marker path (Marker::Match: cv::ORB 2.4 HARRIS 500 features on
    # the frame, BruteForceMatcher<HammingLUT> against the target's descriptors, good filter)
    "AR": dict(w=640, h=480, nfeatures=500, marker=True,
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
        # two launches (levels 1-3 from the input, 4-7 from level 3): average launch
        "k_pyramid": (2 * P[0] * n_img + sum(per_resize)) / 2,
        "k_blur": 2 * sum(P) * n_img,
        "k_fast_tile": sum(P) * n_img,                          # every level pixel read once
        "k_fast_compact": sum(P) * n_img / 8,                   # 1 NMS bit per pixel
        "k_describe": 60 * n_kp,
        "k_voc_transform": 52 * n_kp,                          # desc in; word, rank, node, weight out
        "k_bowvec": 24 * n_kp,
        "total_per_frame": P[0] + sum(per_resize) / n_img + 3 * sum(P) + 60 * n_kp / n_img,
    }


# bytes per lane of the global loads of the kernels bench.py can name as roofline kernel (the
# staged windows of k_fast_tile and k_cvfast: uint2 per lane); their stores are 8-B bitmap words
# and 1-B survivor scores
LOAD_WIDTH = {"k_fast_tile": 8, "k_cvfast": 8}


def pmc_calibration():
    """profiles/pmc_calibration.json (scripts/pmc_calibrate.py, tools/pmc_calib.hip): counter
    bytes per true byte for streaming loads / stores of each width per lane, measured here."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "pmc_calibration.json")))
    except (OSError, ValueError):
        return None


def pmc_traffic(pmc_dir, kernel):
    """HBM-side bytes per launch of `kernel` from separate rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE, both in KB).  MI355X_MICROARCH.md §HBM: FETCH_SIZE counts L2->fabric
    requests (Infinity-Cache hits included) and reads 1/2 of the bytes of 16-B-per-lane streaming
    loads; other widths are to be calibrated in one's own access pattern, which
    profiles/pmc_calibration.json holds (4- and 8-B loads: also 1/2; stores exact).  Returns
    (bytes, note): FETCH_SIZE x 1024 / read factor of the kernel's load width +
    WRITE_SIZE x 1024 / the 8-B store factor, or the uncorrected sum without a calibration."""
    import csv
    tot = {}
    rel = os.path.relpath(pmc_dir, ROOT) if pmc_dir else None
    for name, counter in (("fetch_size.csv", "FETCH_SIZE"), ("write_size.csv", "WRITE_SIZE")):
        path = os.path.join(pmc_dir, name) if pmc_dir else ""
        if not os.path.exists(path):
            return None, f"no PMC passes for this command ({rel})"
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if r["Kernel_Name"].split("(")[0].endswith("::" + kernel) and r["Counter_Name"] == counter]
        if not vals:
            return None, f"kernel not in the PMC passes ({rel})"
        tot[counter] = sum(vals) / len(vals) * 1024
    cal = pmc_calibration()
    w = LOAD_WIDTH.get(kernel)
    rf = (cal or {}).get("read", {}).get(f"{w}B_per_lane") if w else None
    wf = (cal or {}).get("write", {}).get("8B_per_lane")
    if rf and wf:
        return (round(tot["FETCH_SIZE"] / rf + tot["WRITE_SIZE"] / wf),
                f"FETCH_SIZE*1024/{rf} + WRITE_SIZE*1024/{wf} per launch: rocprofv3 --pmc passes of "
                f"this command ({rel}), corrected by profiles/pmc_calibration.json for {w}-B loads")
    return (round(tot["FETCH_SIZE"] + tot["WRITE_SIZE"]),
            f"uncorrected (FETCH_SIZE+WRITE_SIZE)*1024 per launch ({rel}; no calibration for "
            f"this kernel's access width)")


def pmc_valu(pmc_dir, kernel, avg_launch_us):
    """VALU-issue roofline of `kernel` from the SQ counter pass of this bench command
    (sq_counters.csv: SQ_INSTS_VALU summed over a dispatch's waves).  A wave64 VALU instruction
    occupies its SIMD's VALU for one quad-cycle (SQ_ACTIVE_INST_VALU == SQ_INSTS_VALU on these
    kernels), so the issue floor of a launch is INSTS_VALU * 4 / (1024 SIMDs * 2.4 GHz)."""
    import csv
    path = os.path.join(pmc_dir, "sq_counters.csv")
    if not os.path.exists(path) or not avg_launch_us:
        return None
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"].split("(")[0].endswith("::" + kernel)
            and r["Counter_Name"] == "SQ_INSTS_VALU"]
    if not vals:
        return None
    instr = sum(vals) / len(vals)
    floor_us = instr * 4 / 1024 / 2400.0
    return {"valu_instr_per_launch": round(instr), "issue_floor_us": round(floor_us, 2),
            "frac": round(floor_us / avg_launch_us, 4),
            "note": "integer stencil/popcount work: the VALU issue rate, not HBM, bounds it; "
                    "floor = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz), frac = floor / "
                    "avg_launch_us (" + os.path.relpath(path, ROOT) + ")"}


def cpu_baseline(cfg, seconds):
    """The CPU oracle (orb_oracle.cc restating ORBextractor/ORBmatcher) on this host, 1 thread,
    on consecutive frames of the same synthetic stream: extract + SearchByBoW +
    SearchForTriangulation per frame."""
    from oracle import oracle as O
    from ar_orbslam2_amd import synth
    from ar_orbslam2_amd.pipeline import TUM1_K, fundamental_from_pose
    w, h, nf = cfg["w"], cfg["h"], cfg["nfeatures"]
    p = O.params(nf)
    t = O.tables(p, w, h)
    from ar_orbslam2_amd.vocabulary import complete_tree
    ndesc = sum(10 ** l for l in range(7))
    voc = O.Vocabulary.from_nodes(10, 6, 0, 0, *complete_tree(
        10, 6, np.random.default_rng(42).integers(0, 256, (ndesc, 32), dtype=np.uint8)))
    F = fundamental_from_pose()
    ex, ey = O.epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    stereo = cfg.get("stereo")
    if stereo:
        from ar_orbslam2_amd.stereo import stereo_params
        mb, mbf = stereo_params(*stereo)
        imgs = [synth.stereo_pair(w, h, i, 0) for i in range(16)]
    else:
        base = synth.canvas(w, h, 0)
        imgs = [synth.frame(w, h, i, 0, base) for i in range(64)]

    prev = None
    n = 0
    t0 = time.perf_counter()
    while True:
        img = imgs[n % len(imgs)]
        u_right = None
        if stereo:
            kps, desc, pl, _ = O.extract(img[0], p, want_pyramid=True)
            kr, dr, pr, _ = O.extract(img[1], p, want_pyramid=True)
            u_right = O.stereo_matches(kps, desc, kr, dr, pl, pr, t["scale"], t["inv_scale"],
                                       mb, mbf)[0]
        else:
            kps, desc = O.extract(img, p)
        b = voc.transform(desc, 4)  # Frame::ComputeBoW: BowVector + FeatureVector
        r = np.random.default_rng(n)
        cur = dict(desc=desc, angle=kps["angle"], keys=kps,
                   fv=(b["fv_ids"], b["fv_off"], b["fv_feats"]),
                   valid=(r.random(len(kps)) < 0.6).astype(np.uint8),
                   has_mp=(r.random(len(kps)) < 0.4).astype(np.uint8), u_right=u_right,
                   scale_factors=t["scale"], level_sigma2=t["sigma2"])
        if prev is not None:
            O.search_by_bow_kf_f(prev, dict(cur, valid=None), 0.7, True)
            O.search_for_triangulation(prev, cur, F, ex, ey, False, 0.6, False)
        prev = cur
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 4:
            break
    return dict(value=n / el, unit="frames/s", cores=1, kind="port",
                sample=f"{n} consecutive {w}x{h} synthetic {'stereo ' if stereo else ''}frames, CPU "
                       f"oracle (oracle/*.cc, g++ -O3 -march=x86-64-v3 -ffp-contract=off), 1 thread, "
                       f"extract{' x2 + ComputeStereoMatches' if stereo else ''} + "
                       f"ComputeBoW + SearchByBoW + SearchForTriangulation per frame, {el:.1f} s on "
                       f"{platform.processor() or platform.machine()}")


def cpu_baseline_marker(cfg, seconds, target_desc):
    """The CPU oracle of the marker path (cvorb_oracle.cc), 1 thread: cv::ORB of the frame,
    BruteForceMatcher match against the target, Marker::Match's good filter, per frame."""
    from oracle import oracle as O
    from ar_orbslam2_amd import synth
    w, h = cfg["w"], cfg["h"]
    base = synth.canvas(w, h, 0)
    imgs = [synth.frame(w, h, i, 0, base) for i in range(32)]
    p = O.cvorb_params(cfg["nfeatures"])
    n = 0
    t0 = time.perf_counter()
    while True:
        kps, desc = O.cvorb_detect(imgs[n % len(imgs)], p)
        O.good_matches(O.bf_match(target_desc, desc))
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 4:
            break
    return dict(value=n / el, unit="frames/s", cores=1, kind="port",
                sample=f"{n} consecutive {w}x{h} synthetic frames, CPU oracle (oracle/cvorb_oracle.cc, "
                       f"g++ -O3 -march=x86-64-v3 -ffp-contract=off), 1 thread, cv::ORB + "
                       f"BruteForceMatcher vs {len(target_desc)} target descriptors + good filter "
                       f"per frame, {el:.1f} s on {platform.processor() or platform.machine()}")


def marker_bytes(levels, n_kp, n_img, n_target):
    """Algorithmic bytes per launch of the marker-path kernels (same byte model as §8d; the
    matcher reads both descriptor sets once per frame)."""
    P = [w * h for w, h in levels]
    per_resize = [(P[l - 1] + P[l]) * n_img for l in range(1, len(P))]
    return {"k_pyramid": (2 * P[0] * n_img + sum(per_resize)) / 2,
            "k_cvfast": sum(P) * n_img, "k_blur": 2 * sum(P) * n_img,
            "k_cvselect": sum(P) * n_img / 8 + 8 * n_kp, "k_cvdescribe": 60 * n_kp,
            "k_bfmatch": 32 * (n_kp + n_target * n_img) + 8 * n_target * n_img,
            "k_good": 24 * n_target * n_img}


def run_marker(args, cfg, rank, world, local):
    import torch
    from oracle import oracle as O  # the target's descriptors only (fixed input, untimed)
    from ar_orbslam2_amd import synth
    from ar_orbslam2_amd.marker import MarkerBatch
    w, h, nf, B = cfg["w"], cfg["h"], cfg["nfeatures"], args.batch
    S = max(1, args.streams)
    target = synth.frame(w, h, 5, 0)
    _, target_desc = O.cvorb_detect(target, O.cvorb_params(nf))
    pipes, pools = [], []
    for si in range(S):
        mb = MarkerBatch(w, h, B, nf, device=local)
        mb.set_target(target_desc)
        stream_id = stream_of_rank(rank) * S + si
        base = synth.canvas(w, h, stream=stream_id)
        pool = []
        for pi in range(args.pool):
            fr = np.stack([synth.frame(w, h, pi * B + i, stream_id, base) for i in range(B)])
            pool.append(torch.from_numpy(fr).cuda())
        pipes.append(mb)
        pools.append(pool)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
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
    stages = {}
    pipe = pipes[0]
    if not args.no_profile:
        pipe.profile(True)
        for i in range(args.roofline_steps):
            pipe.run(pools[0][i % len(pools[0])].data_ptr(), B)
        pipe.sync()
        stages = pipe.profile_read()
        pipe.profile(False)
    kp_counts, good_counts = pipe.results(B)
    if (kp_counts < 0).any():
        raise RuntimeError("a frame overflowed the per-level keypoint capacity")
    elapsed = aggregate_elapsed(elapsed, world)
    value = world * S * B * args.steps / elapsed
    from ar_orbslam2_amd.marker import cvorb_params
    lv = O.cvorb_levels(cvorb_params(nf), w, h)
    levels = list(zip(lv["w"].tolist(), lv["h"].tolist()))
    n_kp = int(kp_counts.sum())
    alg = marker_bytes(levels, n_kp, B, len(target_desc))
    roofline = None
    if stages:
        dom = max(stages, key=lambda k: stages[k][0])
        ms, launches = stages[dom]
        avg_s = ms / 1e3 / max(launches, 1)
        a_bytes = alg.get(dom)
        achieved = a_bytes / avg_s / 1e9
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 3),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6),
                    "traffic": pmc_traffic(args.pmc_dir, dom)[0],
                    "traffic_note": pmc_traffic(args.pmc_dir, dom)[1],
                    "avg_launch_us": round(avg_s * 1e6, 2),
                    "algorithmic_bytes_per_launch": a_bytes,
                    "valu_roofline": pmc_valu(args.pmc_dir, dom, avg_s * 1e6),
                    "stages_ms_per_step": {k: round(v[0] / args.roofline_steps, 4)
                                           for k, v in stages.items()},
                    "stages_of": f"roofline pass: camera stream 0 alone, {args.roofline_steps} "
                                 f"steps of {B} frames after the timed region"}
    out = {
        "metric": MARKER_METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "frames_per_step_per_gpu": B * S,
                   "camera_streams_per_gpu": S, "frames_per_batch": B, "image": f"{w}x{h}",
                   "nfeatures": nf, "target_descriptors": len(target_desc),
                   "parallelism": f"{world} GPU(s) x {S} independent camera streams, no collective",
                   "keypoints_per_frame": round(n_kp / B, 1),
                   "good_matches_per_frame": round(float(good_counts.mean()), 1),
                   "hamming_pairs_per_frame": round(n_kp / B * len(target_desc)),
                   "timing": "hipGraph replay of the extraction + 2 matcher launches per batch"},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_marker(cfg, args.cpu_seconds, target_desc)
    if rank == 0:
        print(json.dumps(out), flush=True)


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


def stream_of_rank(rank):
    """Camera stream s is processed by rank s (streams shard with no exchange)."""
    return rank


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256,
                    help="frames per step per camera stream")
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--pool", type=int, default=4, help="distinct resident batches cycled")
    ap.add_argument("--streams", type=int, default=3,
                    help="independent camera-stream pipelines per GPU, one HIP stream each "
                         "(kernels are latency-bound; concurrent streams fill the CUs the others leave idle)")
    ap.add_argument("--pmc-dir", default=None,
                    help="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs of this bench command, used "
                         "for roofline.traffic (per launch of the dominant kernel)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the per-kernel roofline pass after the timed region")
    ap.add_argument("--roofline-steps", type=int, default=5,
                    help="steps of the single-stream roofline pass (per-kernel HIP events)")
    args = ap.parse_args()
    if args.pmc_dir is None:  # the committed PMC passes of this config's default command
        # (never another config's: a missing directory reports traffic / VALU floor as null)
        args.pmc_dir = os.path.join(ROOT, "profiles",
                                    "r01_pmc" if args.config == "C2" else
                                    "r01_pmc_" + args.config.lower())

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))

    cfg = CONFIGS[args.config]
    if cfg.get("marker"):
        run_marker(args, cfg, rank, world, local)
        if world > 1:
            dist.destroy_process_group()
        return

    from ar_orbslam2_amd import ORBextractor, Vocabulary, epipole, synth
    from ar_orbslam2_amd.pipeline import TUM1_K, FramePipeline, fundamental_from_pose

    w, h, nf, B = cfg["w"], cfg["h"], cfg["nfeatures"], args.batch
    voc = Vocabulary.synthetic()
    S = max(1, args.streams)
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    pipes, pools = [], []
    stereo = None
    if cfg.get("stereo"):
        from ar_orbslam2_amd.stereo import stereo_params
        stereo = stereo_params(*cfg["stereo"])
    for si in range(S):
        pipe = FramePipeline(w, h, B, voc, nf, device=local, stereo=stereo)
        pipe.seeded_masks(range(B))
        pipe.set_matching(fundamental_from_pose(), (ex, ey), bow_ratio=0.7, bow_check_ori=True,
                          tri_ratio=0.6, tri_check_ori=False)
        # synthetic frames of this camera stream, resident in HBM before timing
        stream_id = stream_of_rank(rank) * S + si
        pool = []
        if stereo:
            pairs = [synth.stereo_pair(w, h, t, stream_id) for t in range(min(B, 32))]
            for pi in range(args.pool):  # interleaved (left, right) images
                fr = np.stack([im for i in range(B) for im in pairs[(pi * 7 + i) % len(pairs)]])
                pool.append(torch.from_numpy(fr).cuda())
        else:
            base = synth.canvas(w, h, stream=stream_id)
            for pi in range(args.pool):
                fr = np.stack([synth.frame(w, h, pi * B + i, stream_id, base) for i in range(B)])
                pool.append(torch.from_numpy(fr).cuda())
        pipes.append(pipe)
        pools.append(pool)
    pipe = pipes[0]
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for i in range(args.warmup):
        for p, pool in zip(pipes, pools):
            p.run(pool[i % len(pool)].data_ptr(), B)
    for p in pipes:
        p.sync()
        if p.results(B)[3]:
            raise RuntimeError("matcher reported a node larger than its per-wave capacity")

    # timed region: every camera stream replays its captured hipGraph, no per-kernel events
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
    # roofline pass (after timing): stream 0 alone with HIP events around every kernel on the
    # stream it launches on, so a kernel's event interval is its own duration (as rocprofv3
    # reports it) rather than a share of the concurrent streams
    stages = {}
    if not args.no_profile:
        pipe.profile(True)
        for i in range(args.roofline_steps):
            pipe.run(pools[0][i % len(pools[0])].data_ptr(), B)
        pipe.sync()
        stages = pipe.profile_read()
        pipe.profile(False)
    kp_counts, bow, tri, _ = pipe.results(B)

    elapsed = aggregate_elapsed(elapsed, world)

    frames = world * S * B * args.steps
    value = frames / elapsed
    ex_tables = ORBextractor(nf)
    levels = level_sizes(w, h, ex_tables.GetInverseScaleFactors())
    n_kp = int(kp_counts.sum())
    # stereo: both images of a frame are extracted (right keypoint count ~ left)
    alg = algorithmic_bytes(levels, 2 * n_kp if stereo else n_kp, 2 * B if stereo else B)
    roofline = None
    if stages:
        dom = max(stages, key=lambda k: stages[k][0])
        ms, launches = stages[dom]
        avg_s = ms / 1e3 / max(launches, 1)
        a_bytes = alg.get(dom)
        achieved = (a_bytes / avg_s / 1e9) if a_bytes is not None else None
        roofline = {"bound": "hbm", "kernel": dom,
                    "achieved": round(achieved, 3) if achieved is not None else None,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6) if achieved is not None else None,
                    "traffic": pmc_traffic(args.pmc_dir, dom)[0],
                    "traffic_note": pmc_traffic(args.pmc_dir, dom)[1],
                    "avg_launch_us": round(avg_s * 1e6, 2),
                    "algorithmic_bytes_per_launch": a_bytes,
                    "valu_roofline": pmc_valu(args.pmc_dir, dom, avg_s * 1e6),
                    "stages_ms_per_step": {k: round(v[0] / args.roofline_steps, 4)
                                           for k, v in stages.items()},
                    "stages_of": f"roofline pass: camera stream 0 alone, {args.roofline_steps} "
                                 f"steps of {B} frames after the timed region"}

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "frames_per_step_per_gpu": B * S,
                   "camera_streams_per_gpu": S, "frames_per_batch": B,
                   "image": f"{w}x{h}", "images_per_frame": 2 if stereo else 1,
                   "nfeatures": nf, "nlevels": 8, "scale_factor": 1.2,
                   "parallelism": f"{world} GPU(s) x {S} independent camera streams, no collective",
                   "keypoints_per_frame": round(n_kp / B, 1),
                   "bow_matches_per_frame": round(float(bow.mean()), 1),
                   "triangulation_matches_per_frame": round(float(tri.mean()), 1),
                   "timing": "hipGraph replay; per-kernel HIP events only in the roofline pass"},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
