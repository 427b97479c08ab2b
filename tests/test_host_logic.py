"""Host-side logic of the mirrors and of the matcher semantics, on the CPU oracle with
hand-built inputs (ORBmatcher.cc rules of SURVEY §8a M1-M5)."""
import json

import numpy as np
import pytest

from ar_orbslam2_amd import FeatureVector, synth
from ar_orbslam2_amd.vocabulary import complete_tree
from oracle import oracle as O


def test_featurevector_from_nodes_is_dbow2_addfeature():
    nodes = np.array([30, 11, 30, 12, 11, 30], np.uint32)
    fv = FeatureVector.from_nodes(nodes)
    assert fv.node_ids.tolist() == [11, 12, 30]
    assert fv.node_offsets.tolist() == [0, 2, 3, 6]
    assert fv.node_feats.tolist() == [1, 4, 3, 0, 2, 5]
    # stopped words (weight <= 0) are not added
    fv = FeatureVector.from_nodes(np.array([30, 0xFFFFFFFF, 11], np.uint32))
    assert fv.node_ids.tolist() == [11, 30] and fv.node_feats.tolist() == [2, 0]


def test_complete_tree_breadth_first_layout():
    desc = np.arange(1111 * 32, dtype=np.uint32).astype(np.uint8).reshape(1111, 32)
    parent, is_leaf, d, w = complete_tree(10, 3, desc)
    assert len(parent) == 1110
    assert parent[:10].tolist() == [0] * 10                     # level 1: ids 1..10
    assert parent[10:20].tolist() == [1] * 10 and parent[109] == 10  # level 2: ids 11..110
    assert parent[110] == 11 and parent[1109] == 110            # level 3: ids 111..1110
    assert is_leaf.sum() == 1000 and is_leaf[110:].all() and not is_leaf[:110].any()
    assert np.array_equal(d, desc[1:]) and (w[110:] == 1.0).all() and (w[:110] == 0).all()


def test_feature_vector_descent_first_child_wins():
    voc = np.zeros((111, 32), np.uint8)  # all nodes identical: ties -> first child
    d = np.random.default_rng(0).integers(0, 256, (5, 32), dtype=np.uint8)
    assert O.feature_vector(voc, 10, 6, 4, d).tolist() == [11] * 5
    assert O.feature_vector(voc, 10, 6, 6, d).tolist() == [0] * 5  # nid_level <= 0 -> root


def _desc(bits):
    d = np.zeros(32, np.uint8)
    for b in bits:
        d[b // 8] |= 1 << (b % 8)
    return d


def _side(descs, angles, nodes, valid=None):
    descs = np.array(descs, np.uint8).reshape(-1, 32)
    fv = FeatureVector.from_nodes(np.array(nodes, np.uint32))
    return dict(desc=descs, angle=np.array(angles, np.float32), valid=valid, fv=fv.as_tuple())


def test_descriptor_distance_is_popcount():
    a, b = _desc([0, 5, 200]), _desc([5, 255])
    assert O.descriptor_distance(a, b) == 3


def test_bow_greedy_skip_and_threshold():
    # two KF features both nearest to F0; the first takes it, the second falls to F1
    f = _side([_desc(range(0, 10)), _desc(range(0, 30))], [0, 0], [11, 11])
    kf = _side([_desc(range(0, 10)), _desc(range(0, 11))], [0, 0], [11, 11], np.array([1, 1], np.uint8))
    n, m = O.search_by_bow_kf_f(kf, f, 0.9, False)
    # KF0: d(F0)=0, d(F1)=20 -> match F0.  KF1: F0 already matched; d(F1)=19, best2=256 -> match
    assert m.tolist() == [0, 1] and n == 2


def test_bow_threshold_le_vs_lt():
    base = _desc([])
    far = _desc(range(50))   # distance exactly 50
    f = _side([far], [0], [11])
    kf = _side([base], [0], [11], np.array([1], np.uint8))
    n1, _ = O.search_by_bow_kf_f(kf, f, 0.99, False)       # KF->Frame accepts <= 50
    n2, _ = O.search_by_bow_kf_kf(dict(kf), dict(f, valid=np.array([1], np.uint8)), 0.99, False)
    assert n1 == 1 and n2 == 0                               # KF->KF needs < 50


def test_bow_invalid_mappoints_are_skipped():
    f = _side([_desc([1])], [0], [11])
    kf = _side([_desc([1])], [0], [11], np.array([0], np.uint8))
    assert O.search_by_bow_kf_f(kf, f, 0.9, False)[0] == 0


def test_rotation_bins_and_three_maxima():
    # 10 matches rotated 0 deg, 2 at 90 deg (bin 3), 1 at 300 deg (bin 10): max1=10, max2=2
    # 2 >= 0.1*10 keeps bin 3, 1 >= 1.0 keeps bin 10 -> nothing removed
    n = 13
    descs = [_desc([i, 100 + i]) for i in range(n)]
    ang_f = [0.0] * n
    ang_kf = [0.0] * 10 + [90.0, 90.0, 300.0]
    f = _side(descs, ang_f, list(range(11, 11 + n)))
    kf = _side(descs, ang_kf, list(range(11, 11 + n)), np.ones(n, np.uint8))
    cnt, m = O.search_by_bow_kf_f(kf, f, 0.9, True)
    assert cnt == 13
    # with 30 at 0 deg the lone 300-deg match (1 < 0.1*30) is dropped, bin 3 (2 < 3) too
    n = 33
    descs = [_desc([i, 100 + i]) for i in range(n)]
    f = _side(descs, [0.0] * n, list(range(11, 11 + n)))
    kf = _side(descs, [0.0] * 30 + [90.0, 90.0, 300.0], list(range(11, 11 + n)), np.ones(n, np.uint8))
    cnt, m = O.search_by_bow_kf_f(kf, f, 0.9, True)
    assert cnt == 30 and (m[30:] == -1).all()


def test_triangulation_last_equal_distance_wins():
    kp = np.zeros(3, O.KEYPOINT_DTYPE)
    kp["x"] = [10, 20, 30]
    kp["y"] = [10, 10, 10]
    d = [_desc([1, 2]), _desc([1]), _desc([2])]  # KF2 features 1 and 2 both at distance 1
    t = O.tables()
    k1 = dict(desc=np.array([d[0]]), keys=kp[:1], u_right=None, has_mp=None,
              fv=FeatureVector.from_nodes(np.array([11], np.uint32)).as_tuple(),
              scale_factors=t["scale"], level_sigma2=t["sigma2"])
    k2 = dict(desc=np.array(d), keys=kp, u_right=None, has_mp=np.array([1, 0, 0], np.uint8),
              fv=FeatureVector.from_nodes(np.array([11, 11, 11], np.uint32)).as_tuple(),
              scale_factors=t["scale"], level_sigma2=t["sigma2"])
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)  # horizontal epipolar lines
    n, pairs = O.search_for_triangulation(k1, k2, F, 1e6, 1e6, False, 0.6, False)
    assert n == 1 and pairs.tolist() == [[0, 2]]


def test_synthetic_frames_are_deterministic():
    a = synth.frame(64, 48, t=3, stream=1)
    b = synth.frame(64, 48, t=3, stream=1)
    assert np.array_equal(a, b) and a.dtype == np.uint8 and a.shape == (48, 64)


def test_bench_extract_vs_match_split():
    """bench.py's §8d phase split: extraction stages vs matcher stages of the roofline pass."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    st = {"k_pyramid": (1.0, 5), "k_fast_cells": (2.0, 5), "k_describe": (1.0, 5),
          "k_voc_transform": (0.5, 5), "k_bow": (0.5, 5), "k_stereo": (1.0, 5)}
    s = bench.phase_split(st, 5, 256)
    assert s["extract_ms_per_batch"] == pytest.approx(0.8)
    assert s["match_ms_per_batch"] == pytest.approx(0.4)
    assert s["combined_frames_per_s_one_stream"] == pytest.approx(256 / 1.2e-3, rel=1e-6)
    assert s["match_stages"] == ["k_bow", "k_stereo", "k_voc_transform"]


def test_summarizer_finds_roofline_pass(tmp_path):
    """scripts/summarize_profiles.py: the roofline pass is the longest run of dispatches on one
    stream that no other stream's dispatch overlaps (the timed region and the PCIe pass run the
    camera streams concurrently; the timed region's tail may leave one stream's last dispatches
    in a row, overlapped by the others' — the round-5 C5 trace did)."""
    import csv
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                        "summarize_profiles.py")
    spec = importlib.util.spec_from_file_location("summarize_profiles", path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    timed = [(700, s, False) for _ in range(4) for s in "123"]
    tail = [(900, "1", False) for _ in range(6)]  # stream 1 ahead, the others still running
    solo = [(650 + i, "1", True) for i in range(5)]
    pcie = [(720, s, False) for _ in range(3) for s in "123"]
    assert m.solo_run(timed + tail + solo + pcie) == [650, 651, 652, 653, 654]
    assert m.solo_run(timed) == [700] * 5  # no solo run: the last dispatches
    # the overlap test on a trace: k on stream 1 overlapped by stream 2's dispatch, then alone
    rows = [("k", 0, 100, "1"), ("j", 50, 150, "2"), ("k", 200, 300, "1"), ("k", 300, 400, "1")]
    f = tmp_path / "t.csv"
    with open(f, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"])
        w.writerows(rows)
    d = m.trace_durations(str(f))
    assert d["k"] == [(100, "1", False), (100, "1", True), (100, "1", True)]


def test_pmc_compaction_keeps_bench_readings(tmp_path, monkeypatch):
    """scripts/pmc_compact.py rewrites a --pmc pass to one row per (kernel, counter) holding the
    mean per dispatch: bench.py's traffic and issue readings and the summarizer's per-dispatch
    sums are unchanged (the committed round-3 passes are compact)."""
    import csv
    import importlib.util
    import os
    import shutil
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = []
    for d, (kn, vals) in enumerate([("void orbx::k_fast_cells<44, 44, unsigned int>(x)", (10., 14.)),
                                    ("void orbx::k_fast_cells<72, 66, unsigned int>(x)", (2., 4.)),
                                    ("orbx::k_blur(x)", (7., 9.))]):
        for i, v in enumerate(vals):
            for c, scale in (("FETCH_SIZE", 1.0), ("WRITE_SIZE", 0.5)):
                rows.append({"Dispatch_Id": str(10 * d + i), "Kernel_Name": kn, "Counter_Name": c,
                             "Counter_Value": str(v * scale)})
    full, comp = tmp_path / "full", tmp_path / "comp"
    full.mkdir()
    for name, c in (("fetch_size.csv", "FETCH_SIZE"), ("write_size.csv", "WRITE_SIZE")):
        with open(full / name, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(r for r in rows if r["Counter_Name"] == c)
    shutil.copytree(full, comp)
    spec = importlib.util.spec_from_file_location("pmc_compact", os.path.join(root, "scripts", "pmc_compact.py"))
    pc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pc)
    pc.compact(str(comp / "fetch_size.csv"))
    pc.compact(str(comp / "write_size.csv"))
    assert len(list(csv.DictReader(open(comp / "fetch_size.csv")))) == 3
    sys.path.insert(0, root)
    import bench
    inst = ["k_fast_cells<44, 44, unsigned int>", "k_fast_cells<72, 66, unsigned int>"]
    for d in (full, comp):
        (d / "meta.json").write_text(json.dumps({"lib_srchash": "h0", "kernels": inst + ["k_blur"]}))
    monkeypatch.setattr(bench, "library_hash", lambda: ("h0", False, root))
    tf, tc = bench.pmc_traffic(str(full), inst)[0], bench.pmc_traffic(str(comp), inst)[0]
    assert tf is not None and tf == tc
    spec = importlib.util.spec_from_file_location("summarize_profiles",
                                                  os.path.join(root, "scripts", "summarize_profiles.py"))
    sm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sm)
    a1, c1 = sm.counters(str(full))
    a2, c2 = sm.counters(str(comp))
    for k in a1:
        for c in a1[k]:
            assert a1[k][c] == pytest.approx(a2[k][c]) and len(c1[(k, c)]) == len(c2[(k, c)])


def test_roofline_bytes_split_over_a_stages_dispatches():
    """bench.py's algorithmic bytes are per step; a stage with several dispatches per step (the
    pyramid: one per pyramid stage) gets them split over its launches, as avg_launch_us and the
    PMC readers (mean per dispatch) are per launch; with the blur fused (no k_blur stage) the
    blur's bytes count under k_pyramid."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    alg = {"k_pyramid": 600.0, "k_blur": 300.0, "k_describe": 10.0}
    # 5 steps, 3 pyramid dispatches each, 2 ms in total: 15 launches of 2/15 ms
    st = {"k_pyramid": (2.0, 15), "k_describe": (0.5, 5)}
    r = bench.roofline_of(st, alg, None, 5, 512)
    assert r["kernel"] == "k_pyramid" and r["launches_per_step"] == 3.0
    assert r["algorithmic_bytes_per_launch"] == pytest.approx(900.0 / 3)
    assert r["avg_launch_us"] == pytest.approx(2000.0 / 15, rel=1e-3)
    # separate blur: the pyramid's own bytes only
    st = {"k_pyramid": (2.0, 10), "k_blur": (1.0, 5), "k_describe": (0.5, 5)}
    r = bench.roofline_of(st, alg, None, 5, 512)
    assert r["algorithmic_bytes_per_launch"] == pytest.approx(600.0 / 2)


def test_pmc_fields_bound_to_library_and_instances(tmp_path, monkeypatch):
    """bench.py's counter fields (roofline.traffic, issue_roofline) come only from PMC passes of
    the library build that ran (meta.json's lib_srchash) and only from the exact kernel
    instances the roofline pass launched for the stage: k_pyramid<true> never reads
    k_pyramid<false>'s (or another build's) counters; otherwise the fields are null with the
    reason."""
    import csv
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    d = tmp_path / "pmc"
    d.mkdir()
    names = {"void orbx::k_pyramid<false>(unsigned char const*)": 100.0,
             "void orbx::k_pyramid<true>(unsigned char const*)": 300.0}
    for fn, c in (("fetch_size.csv", "FETCH_SIZE"), ("write_size.csv", "WRITE_SIZE")):
        with open(d / fn, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "Dispatches"])
            for k, v in names.items():
                w.writerow([k, c, v, 3])
    with open(d / "sq_counters.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "Dispatches"])
        for k, v in names.items():
            for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_SALU"):
                w.writerow([k, c, v * (0 if c.endswith("VALU2") else 1000), 3])
    (d / "meta.json").write_text(json.dumps({"lib_srchash": "abc",
                                             "kernels": ["k_pyramid<false>", "k_pyramid<true>"]}))
    monkeypatch.setattr(bench, "library_hash", lambda: ("abc", False, root))
    t_true, _ = bench.pmc_traffic(str(d), ["k_pyramid<true>"])
    t_false, _ = bench.pmc_traffic(str(d), ["k_pyramid<false>"])
    assert t_true is not None and t_false is not None and t_true == 3 * t_false
    it = bench.pmc_issue(str(d), ["k_pyramid<true>"], 100.0)
    iff = bench.pmc_issue(str(d), ["k_pyramid<false>"], 100.0)
    assert it["valu_instr_per_launch"] == 300000 and iff["valu_instr_per_launch"] == 100000
    # an instance the passes do not hold: null, with the reason
    t, why = bench.pmc_traffic(str(d), ["k_fast_pairs<unsigned int>"])
    assert t is None and "k_fast_pairs<unsigned int>" in why
    assert bench.pmc_issue(str(d), ["k_fast_pairs<unsigned int>"], 100.0)["frac"] is None
    # passes of another build: null, with the reason
    monkeypatch.setattr(bench, "library_hash", lambda: ("other", False, root))
    t, why = bench.pmc_traffic(str(d), ["k_pyramid<true>"])
    assert t is None and "another library build" in why
    assert bench.pmc_issue(str(d), ["k_pyramid<true>"], 100.0)["frac"] is None
    # no meta.json: not bound to a build
    (d / "meta.json").unlink()
    monkeypatch.setattr(bench, "library_hash", lambda: ("abc", False, root))
    t, why = bench.pmc_traffic(str(d), ["k_pyramid<true>"])
    assert t is None and "meta.json" in why
    # roofline_of carries the instances and nulls the counter fields
    r = bench.roofline_of({"k_pyramid": (2.0, 15)}, {"k_pyramid": 600.0}, str(d), 5, 512,
                          {"k_pyramid": ["k_pyramid<true>"]})
    assert r["kernel_instances"] == ["k_pyramid<true>"] and r["traffic"] is None
    assert r["issue_roofline"]["frac"] is None


def test_kernel_instance_names():
    """rocprofv3 Kernel_Name -> the library profiler's instance name."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    ki = bench.kernel_instance
    assert ki("void orbx::k_fast_cells<44, 42, unsigned int>(unsigned char const*, long)") == \
        "k_fast_cells<44, 42, unsigned int>"
    assert ki("void orbx::k_octree<1024, unsigned long>(orbx::LevelGeom const*, int)") == \
        "k_octree<1024, unsigned long>"
    assert ki("orbx::k_tri_nodes(orbx::TriProblem const*)") == "k_tri_nodes"
    assert ki("(anonymous namespace)::k_fill_u32(unsigned int*, unsigned long)") == "k_fill_u32"


def test_roofline_bytes_follow_survey_8d():
    """The per-kernel algorithmic bytes add up to SURVEY §8d's B per image (4,788,674 B at
    C1/C2), with the input counted once; the level-0 write of the pitched pyramid is carried
    beside it as the builder's model and never enters `frac`."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    levels = bench.level_sizes(640, 480, [1 / 1.2 ** l for l in range(8)])
    alg = bench.algorithmic_bytes(levels, 1000, 1)
    assert alg["k_pyramid"] + alg["k_blur"] + alg["k_fast_cells"] + alg["k_describe"] == 4788674
    assert alg["total_per_frame"] == 4788674
    st = {"k_pyramid": (3.0, 3)}
    r = bench.roofline_of(st, alg, None, 1, 1)
    assert r["algorithmic_bytes_per_launch"] == pytest.approx((alg["k_pyramid"] + alg["k_blur"]) / 3)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS, abs=1e-6)
    b = r["builder_model"]
    assert b["algorithmic_bytes_per_launch"] == pytest.approx(r["algorithmic_bytes_per_launch"] + 307200 / 3)
    assert b["frac"] > r["frac"]
