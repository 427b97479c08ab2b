"""GPU parity of the device frame pipeline (bench.py's unit of work) against the CPU oracle:
per-frame keypoints/descriptors, node ids, SearchByBoW matches and SearchForTriangulation
pairs for a small batch, frame f matched against frame (f-1) mod n."""
import ctypes as C

import numpy as np
import pytest
import torch

from ar_orbslam2_amd import KEYPOINT_DTYPE, Vocabulary, epipole, synth
from ar_orbslam2_amd.vocabulary import complete_tree
from ar_orbslam2_amd.pipeline import TUM1_K, FramePipeline, fundamental_from_pose
from oracle import oracle as O

from matchdata import featvec

pytestmark = pytest.mark.gpu

_hip = None


def d2h(ptr, nbytes):
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
    out = np.zeros(nbytes, np.uint8)
    rc = _hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr), C.c_size_t(nbytes), 2)
    assert rc == 0
    return out


_VOCS = []


def _vocabs():
    """The bench vocabulary (complete k=10, L=6, seed 42) on the GPU and in the oracle."""
    if not _VOCS:
        n = sum(10 ** l for l in range(7))
        desc = np.random.default_rng(42).integers(0, 256, (n, 32), dtype=np.uint8)
        arrays = complete_tree(10, 6, desc)
        _VOCS.append((Vocabulary.from_nodes(10, 6, 0, 0, *arrays),
                      O.Vocabulary.from_nodes(10, 6, 0, 0, *arrays)))
    return _VOCS[0]


@pytest.mark.parametrize("w,h,nf,n", [(640, 480, 1000, 4), (752, 480, 1200, 3),
                                      (1920, 1080, 4000, 2)])
def test_pipeline_matches_oracle(w, h, nf, n):
    voc, oracle_voc = _vocabs()
    pipe = FramePipeline(w, h, n, voc, nf)
    valid, has_mp = pipe.seeded_masks(range(n))
    F = fundamental_from_pose()
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    pipe.set_matching(F, (ex, ey), bow_ratio=0.7, bow_check_ori=True, tri_ratio=0.6,
                      tri_check_ori=False)
    frames = synth.frames(w, h, n, stream=2)
    d = torch.from_numpy(frames).cuda()
    pipe.run(d.data_ptr(), n)
    pipe.run(d.data_ptr(), n)  # second run replays the captured graph
    pipe.sync()
    counts, bow, tri, err = pipe.results(n)
    assert err == 0
    cap = pipe.kp_cap
    out = pipe.device_outputs()
    kps_all = d2h(out["kps"], n * cap * 28).view(KEYPOINT_DTYPE).reshape(n, cap)
    desc_all = d2h(out["desc"], n * cap * 32).reshape(n, cap, 32)
    nodes_all = d2h(out["node_of"], n * cap * 4).view(np.uint32).reshape(n, cap)
    bo = pipe.bow_outputs()
    words_all = d2h(bo["bow_words"], n * cap * 4).view(np.uint32).reshape(n, cap)
    vals_all = d2h(bo["bow_values"], n * cap * 8).view(np.float64).reshape(n, cap)
    nw_all = d2h(bo["bow_n"], n * 4).view(np.int32)
    word_of_all = d2h(bo["word_of"], n * cap * 4).view(np.uint32).reshape(n, cap)
    match_all = d2h(out["bow_match"], n * cap * 4).view(np.int32).reshape(n, cap)
    pairs_all = d2h(out["tri_pairs"], n * cap * 8).view(np.int32).reshape(n, cap, 2)
    t = O.tables(O.params(nf), w, h)
    ref = []
    for f in range(n):
        kps, desc = O.extract(frames[f], O.params(nf))
        k = len(kps)
        assert counts[f] == k
        assert np.array_equal(kps_all[f, :k], kps)
        assert np.array_equal(desc_all[f, :k], desc)
        r = oracle_voc.transform(desc, 4)  # Frame::ComputeBoW
        nodes = r["node_of"]
        assert np.array_equal(nodes_all[f, :k], nodes)
        assert np.array_equal(word_of_all[f, :k], r["word_of"])
        assert nw_all[f] == len(r["bow_words"])
        assert np.array_equal(words_all[f, :nw_all[f]], r["bow_words"])
        assert np.array_equal(vals_all[f, :nw_all[f]], r["bow_values"])  # bit-exact f64
        ref.append(dict(desc=desc, angle=kps["angle"], keys=kps, fv=featvec(nodes),
                        valid=valid[f, :k], has_mp=has_mp[f, :k], scale_factors=t["scale"],
                        level_sigma2=t["sigma2"]))
    for f in range(n):
        kf, cur = ref[(f - 1) % n], ref[f]
        nb, mb = O.search_by_bow_kf_f(kf, dict(cur, valid=None), 0.7, True)
        assert bow[f] == nb
        assert np.array_equal(match_all[f, :len(cur["desc"])], mb)
        nt, pt = O.search_for_triangulation(kf, cur, F, ex, ey, False, 0.6, False)
        assert tri[f] == nt
        assert np.array_equal(pairs_all[f, :nt], pt)
    pipe.close()


@pytest.mark.parametrize("w,h,nf,cam,n", [(752, 480, 1200, (47.90639384423901, 435.2046959714599), 3),
                                          (1241, 376, 2000, (386.1448, 718.856), 2)])
def test_stereo_pipeline_matches_oracle(w, h, nf, cam, n):
    """EuRoC / KITTI stereo geometry (SURVEY configs C3 / C4): extraction of both images,
    ComputeStereoMatches, ComputeBoW of the left image, SearchByBoW and SearchForTriangulation
    with mvuRight, frame f against frame (f-1) mod n."""
    from ar_orbslam2_amd.stereo import stereo_params
    mb, mbf = stereo_params(*cam)
    voc, oracle_voc = _vocabs()
    pipe = FramePipeline(w, h, n, voc, nf, stereo=(mb, mbf))
    valid, has_mp = pipe.seeded_masks(range(n))
    F = fundamental_from_pose()
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    pipe.set_matching(F, (ex, ey), bow_ratio=0.7, bow_check_ori=True, tri_ratio=0.6,
                      tri_check_ori=False)
    pairs = [synth.stereo_pair(w, h, t, 5, (10 + 2 * t, 25)) for t in range(n)]
    imgs = np.stack([im for pr in pairs for im in pr])
    d = torch.from_numpy(imgs).cuda()
    pipe.run(d.data_ptr(), n)
    pipe.sync()
    counts, bow, tri, err = pipe.results(n)
    assert err == 0
    cap = pipe.kp_cap
    out = pipe.device_outputs()
    so = pipe.stereo_outputs()
    kps_all = d2h(out["kps"], 2 * n * cap * 28).view(KEYPOINT_DTYPE).reshape(2 * n, cap)
    match_all = d2h(out["bow_match"], n * cap * 4).view(np.int32).reshape(n, cap)
    pairs_all = d2h(out["tri_pairs"], n * cap * 8).view(np.int32).reshape(n, cap, 2)
    ur_all = d2h(so["uright"], n * cap * 4).view(np.float32).reshape(n, cap)
    dp_all = d2h(so["depth"], n * cap * 4).view(np.float32).reshape(n, cap)
    p = O.params(nf)
    t = O.tables(p, w, h)
    ref = []
    for f in range(n):
        kl, dl, pl, _ = O.extract(pairs[f][0], p, want_pyramid=True)
        kr, dr, prr, _ = O.extract(pairs[f][1], p, want_pyramid=True)
        k = len(kl)
        assert counts[f] == k
        assert np.array_equal(kps_all[2 * f, :k], kl)
        assert np.array_equal(kps_all[2 * f + 1, :len(kr)], kr)
        ur, dp, _ = O.stereo_matches(kl, dl, kr, dr, pl, prr, t["scale"], t["inv_scale"], mb, mbf)
        assert ur_all[f, :k].tobytes() == ur.tobytes()
        assert dp_all[f, :k].tobytes() == dp.tobytes()
        assert (ur >= 0).sum() > 100
        r = oracle_voc.transform(dl, 4)
        ref.append(dict(desc=dl, angle=kl["angle"], keys=kl, fv=featvec(r["node_of"]),
                        valid=valid[f, :k], has_mp=has_mp[f, :k], u_right=ur,
                        scale_factors=t["scale"], level_sigma2=t["sigma2"]))
    for f in range(n):
        kf, cur = ref[(f - 1) % n], ref[f]
        nb, mbm = O.search_by_bow_kf_f(kf, dict(cur, valid=None), 0.7, True)
        assert bow[f] == nb
        assert np.array_equal(match_all[f, :len(cur["desc"])], mbm)
        nt, pt = O.search_for_triangulation(kf, cur, F, ex, ey, False, 0.6, False)
        assert tri[f] == nt
        assert np.array_equal(pairs_all[f, :nt], pt)
    pipe.close()


def test_large_batch_graph_replay_c5():
    """C5 geometry (1920x1080, 4000 features) at a batch whose per-batch match arrays exceed
    512 KiB, replayed from the captured hipGraph: the match arrays are pre-filled with -1 inside
    the graph (a captured memset node of that size once left stale indices behind and the
    rotation filter then read out of bounds).  Frames 0, 1 and n-1 are checked against the
    oracle (frame 0 is matched against frame n-1)."""
    w, h, nf, n = 1920, 1080, 4000, 36
    voc, oracle_voc = _vocabs()
    pipe = FramePipeline(w, h, n, voc, nf)
    valid, has_mp = pipe.seeded_masks(range(n))
    F = fundamental_from_pose()
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    pipe.set_matching(F, (ex, ey), bow_ratio=0.7, bow_check_ori=True, tri_ratio=0.6,
                      tri_check_ori=False)
    base = synth.canvas(w, h, stream=0)
    frames = np.stack([synth.frame(w, h, t, 0, base) for t in range(n)])
    d = torch.from_numpy(frames).cuda()
    for _ in range(3):  # capture, then replays
        pipe.run(d.data_ptr(), n)
    pipe.sync()
    counts, bow, tri, err = pipe.results(n)
    assert err == 0
    cap = pipe.kp_cap
    assert n * cap * 4 > 512 * 1024
    out = pipe.device_outputs()
    match_all = d2h(out["bow_match"], n * cap * 4).view(np.int32).reshape(n, cap)
    pairs_all = d2h(out["tri_pairs"], n * cap * 8).view(np.int32).reshape(n, cap, 2)
    t = O.tables(O.params(nf), w, h)
    ref = {}
    for f in (n - 1, 0, 1):
        kps, desc = O.extract(frames[f], O.params(nf))
        assert counts[f] == len(kps)
        r = oracle_voc.transform(desc, 4)
        ref[f] = dict(desc=desc, angle=kps["angle"], keys=kps, fv=featvec(r["node_of"]),
                      valid=valid[f, :len(kps)], has_mp=has_mp[f, :len(kps)],
                      scale_factors=t["scale"], level_sigma2=t["sigma2"])
    for f in (0, 1):
        kf, cur = ref[(f - 1) % n], ref[f]
        nb, mb = O.search_by_bow_kf_f(kf, dict(cur, valid=None), 0.7, True)
        assert bow[f] == nb
        assert np.array_equal(match_all[f, :len(cur["desc"])], mb)
        nt, pt = O.search_for_triangulation(kf, cur, F, ex, ey, False, 0.6, False)
        assert tri[f] == nt
        assert np.array_equal(pairs_all[f, :nt], pt)
    pipe.close()


@pytest.mark.parametrize("w,h,nf,n", [(1920, 1080, 4000, 6), (640, 480, 1000, 16)])
def test_batch_keypoints_every_frame(w, h, nf, n):
    """Every frame of a batch, keypoints and descriptors bit-exact: the FAST-cell compaction
    and the minThFAST fallback queues (one counter line per image, filled a wave at a time)
    are shared by the whole batch; the 1920x1080 synthetic frames leave ~60 % of their cells
    empty at iniThFAST."""
    voc, _ = _vocabs()
    pipe = FramePipeline(w, h, n, voc, nf)
    pipe.seeded_masks(range(n))
    pipe.set_matching(fundamental_from_pose(), (0.0, 0.0), bow_ratio=0.7, bow_check_ori=True,
                      tri_ratio=0.6, tri_check_ori=False)
    frames = synth.frames(w, h, n, stream=3)
    d = torch.from_numpy(frames).cuda()
    pipe.run(d.data_ptr(), n)
    pipe.run(d.data_ptr(), n)
    pipe.sync()
    counts, _, _, err = pipe.results(n)
    assert err == 0
    cap = pipe.kp_cap
    out = pipe.device_outputs()
    kps_all = d2h(out["kps"], n * cap * 28).view(KEYPOINT_DTYPE).reshape(n, cap)
    desc_all = d2h(out["desc"], n * cap * 32).reshape(n, cap, 32)
    for f in range(n):
        kps, desc = O.extract(frames[f], O.params(nf))
        k = len(kps)
        assert counts[f] == k, f
        assert np.array_equal(kps_all[f, :k], kps), f
        assert np.array_equal(desc_all[f, :k], desc), f
    pipe.close()


_ORACLE_MEMO = {}


def _oracle_extract(img, nf, pyramid=False):
    """O.extract of one image, memoised by content (the stereo pools repeat 32 pairs)."""
    import hashlib
    key = (hashlib.sha1(img.tobytes()).hexdigest(), img.shape, nf, pyramid)
    if key not in _ORACLE_MEMO:
        if len(_ORACLE_MEMO) > 256:
            _ORACLE_MEMO.clear()
        _ORACLE_MEMO[key] = O.extract(img, O.params(nf), want_pyramid=pyramid)
    return _ORACLE_MEMO[key]


def _check_pipe_frames(pipe, frames, which, nf, n, oracle_voc, stereo=None):
    """Frames `which` of the pipeline's last batch (host copy `frames`: n frames, or 2n
    interleaved (left, right) images with `stereo` = (mb, mbf)) against the oracle: keypoints and
    descriptors (both images of a stereo frame), mvuRight / mvDepth (ComputeStereoMatches,
    Frame.cc:471-643), node / word ids, BowVector (f64 bits), SearchByBoW matches and
    SearchForTriangulation pairs with mvuRight (frame f against (f - 1) mod n)."""
    h, w = frames.shape[1:]
    ni = 2 * n if stereo else n
    valid, has_mp = pipe.masks
    ex, ey = pipe.epipole
    F = fundamental_from_pose()
    counts, bow, tri, err = pipe.results(n)
    assert err == 0
    cap = pipe.kp_cap
    out, bo = pipe.device_outputs(), pipe.bow_outputs()
    kps_all = d2h(out["kps"], ni * cap * 28).view(KEYPOINT_DTYPE).reshape(ni, cap)
    desc_all = d2h(out["desc"], ni * cap * 32).reshape(ni, cap, 32)
    nodes_all = d2h(out["node_of"], n * cap * 4).view(np.uint32).reshape(n, cap)
    words_all = d2h(bo["bow_words"], n * cap * 4).view(np.uint32).reshape(n, cap)
    vals_all = d2h(bo["bow_values"], n * cap * 8).view(np.float64).reshape(n, cap)
    nw_all = d2h(bo["bow_n"], n * 4).view(np.int32)
    word_of_all = d2h(bo["word_of"], n * cap * 4).view(np.uint32).reshape(n, cap)
    match_all = d2h(out["bow_match"], n * cap * 4).view(np.int32).reshape(n, cap)
    pairs_all = d2h(out["tri_pairs"], n * cap * 8).view(np.int32).reshape(n, cap, 2)
    if stereo:
        so = pipe.stereo_outputs()
        ur_all = d2h(so["uright"], n * cap * 4).view(np.float32).reshape(n, cap)
        dp_all = d2h(so["depth"], n * cap * 4).view(np.float32).reshape(n, cap)
    t = O.tables(O.params(nf), w, h)
    ref = {}
    for f in sorted(set(which) | {(f - 1) % n for f in which}):
        if stereo:
            kps, desc, pl, _ = _oracle_extract(frames[2 * f], nf, True)
            kr, dr, pr, _ = _oracle_extract(frames[2 * f + 1], nf, True)
            assert np.array_equal(kps_all[2 * f + 1, :len(kr)], kr), f
            assert np.array_equal(desc_all[2 * f + 1, :len(kr)], dr), f
            li = 2 * f
        else:
            kps, desc = _oracle_extract(frames[f], nf)
            li = f
        k = len(kps)
        assert counts[f] == k, f
        assert np.array_equal(kps_all[li, :k], kps), f
        assert np.array_equal(desc_all[li, :k], desc), f
        ur = None
        if stereo:
            ur, dp, _ = O.stereo_matches(kps, desc, kr, dr, pl, pr, t["scale"], t["inv_scale"],
                                         *stereo)
            assert ur_all[f, :k].tobytes() == ur.tobytes(), f
            assert dp_all[f, :k].tobytes() == dp.tobytes(), f
        r = oracle_voc.transform(desc, 4)
        assert np.array_equal(nodes_all[f, :k], r["node_of"]), f
        assert np.array_equal(word_of_all[f, :k], r["word_of"]), f
        assert nw_all[f] == len(r["bow_words"]), f
        assert np.array_equal(words_all[f, :nw_all[f]], r["bow_words"]), f
        assert vals_all[f, :nw_all[f]].tobytes() == r["bow_values"].tobytes(), f
        ref[f] = dict(desc=desc, angle=kps["angle"], keys=kps, fv=featvec(r["node_of"]),
                      valid=valid[f, :k], has_mp=has_mp[f, :k], scale_factors=t["scale"],
                      level_sigma2=t["sigma2"])
        if stereo:
            ref[f]["u_right"] = ur
    for f in which:
        kf, cur = ref[(f - 1) % n], ref[f]
        nb, mb = O.search_by_bow_kf_f(kf, dict(cur, valid=None), 0.7, True)
        assert bow[f] == nb, f
        assert np.array_equal(match_all[f, :len(cur["desc"])], mb), f
        nt, pt = O.search_for_triangulation(kf, cur, F, ex, ey, False, 0.6, False)
        assert tri[f] == nt, f
        assert np.array_equal(pairs_all[f, :nt], pt), f


@pytest.mark.timeout(1100)
@pytest.mark.parametrize("config,argv", [
    ("C2", []),                                                  # 3 streams x 512, pool 4
    ("C3", []),                                                  # 3 streams x 512 stereo pairs
    ("C4", []),                                                  # 3 streams x 512 stereo pairs
    ("C5", []),                                                  # 3 streams x 512
    ("C5", ["--streams-total", "8", "--pool", "2", "--batch", "256"]),  # 8 streams x 256, one GPU
])
def test_bench_timed_topology_matches_oracle(config, argv):
    """bench.py's timed configuration, built by bench's own make_frame_pipes / replay_step, for
    every bench config: C2 / C3 / C4 / C5 at their defaults (three camera streams of 512 frames
    — C3 / C4 frames are (left, right) pairs — a pool of 4 resident batches, every stream's
    captured hipGraphs replayed interleaved across the three HIP streams) and C5's single-GPU
    strong-scaling shape (8 streams of 256 frames).  After the setup captures, the warm-up and 12
    interleaved steps (the compared batch's graph has run 3 times), frames
    {0, 1, 2, 255, 256, 510, 511} (C5 x 256: {0, 1, 2, 127, 128, 254, 255}) of every stream equal
    the oracle: keypoints and descriptors (both images for stereo), mvuRight / mvDepth, BoW,
    SearchByBoW, SearchForTriangulation (Frame.cc:66-122, 471-643)."""
    import bench
    args = bench.parse_args(["--config", config, "--no-upload", "--no-cpu-baseline"] + argv)
    cfg = bench.CONFIGS[config]
    streams = bench.streams_of_rank(0, 1, args.streams, args.streams_total)
    B = args.batch
    pipes, pools, _ = bench.make_frame_pipes(args, cfg, streams, 0)
    print(f"[{config}] pipelines and pools built", flush=True)
    steps = 12
    for i in range(len(pools[0])):
        bench.replay_step(pipes, pools, B, i)
    for i in range(args.warmup):
        bench.replay_step(pipes, pools, B, i)
    for i in range(steps):
        bench.replay_step(pipes, pools, B, i)
    for p in pipes:
        p.sync()
    last = (steps - 1) % len(pools[0])
    which = ([0, 1, 2, 255, 256, 510, 511] if B == 512 else
             [0, 1, 2, B // 2 - 1, B // 2, B - 2, B - 1])
    stereo = None
    if cfg.get("stereo"):
        from ar_orbslam2_amd.stereo import stereo_params
        stereo = stereo_params(*cfg["stereo"])
    _, oracle_voc = _vocabs()
    for si, (p, pool) in enumerate(zip(pipes, pools)):
        frames = pool[last].cpu().numpy()
        _check_pipe_frames(p, frames, which, cfg["nfeatures"], B, oracle_voc, stereo)
        print(f"[{config}] stream {si}: frames {which} equal the oracle", flush=True)
    for p in pipes:
        p.close()
    del pools
    torch.cuda.empty_cache()
