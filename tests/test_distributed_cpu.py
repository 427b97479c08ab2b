"""N>1 path of bench.py on CPU: world_size-2 gloo ranks, each with its own camera streams, the
job time is the max over ranks and the frame count is the sum (no data-path collective).
Drives bench.py's own launcher (`--gpus 2` without WORLD_SIZE), the torchrun launch the driver
uses, and the strong-scaling mode (`--streams-total`), all with `--dry-run` (no device work)."""
import json
import os
import socket
import subprocess
import sys

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from ar_orbslam2_amd import synth
    el = bench.aggregate_elapsed(1.0 + rank, world)
    s = bench.streams_of_rank(rank, world)
    img = synth.frame(64, 48, t=0, stream=s[0])
    q.put((rank, el, s, int(img.sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_aggregation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2.0, 2.0]          # max over ranks
    assert [r[2] for r in res] == [[0], [1]]          # one stream per rank
    assert res[0][3] != res[1][3]                     # independent inputs


def test_stream_sharding():
    import bench
    # weak: G x S streams, s -> GPU s mod G
    assert bench.streams_of_rank(0, 2, 3) == [0, 2, 4]
    assert bench.streams_of_rank(1, 2, 3) == [1, 3, 5]
    # strong: C5's 8 streams over G = 1, 2, 4, 8
    for g in (1, 2, 4, 8):
        parts = [bench.streams_of_rank(r, g, 3, 8) for r in range(g)]
        assert sorted(s for p in parts for s in p) == list(range(8))
        assert all(len(p) == 8 // g for p in parts)
    assert bench.stream_of_rank(1) == 1


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out  # rank 0 only prints
    return json.loads(lines[0])


def test_bench_launcher_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--steps", "3", "--batch", "8"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    per_rank = d["config"]["streams_per_rank"]
    assert per_rank == [[0, 2, 4], [1, 3, 5]]  # distinct streams, 3 per GPU
    assert d["value"] > 0


def test_bench_launcher_strong_scaling():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--streams-total", "8", "--config", "C5", "--steps", "2"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["streams_per_rank"] == [[0, 2, 4, 6], [1, 3, 5, 7]]


def test_bench_under_torchrun():
    """The driver's N>1 launch: torch.distributed.run sets RANK/LOCAL_RANK/WORLD_SIZE."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--steps", "2"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2
    assert d["config"]["streams_per_rank"] == [[0, 2, 4], [1, 3, 5]]


def test_launcher_reports_failing_rank():
    """A rank that fails makes the launcher fail (no silent single-GPU line)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--streams-total", "1"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode != 0
