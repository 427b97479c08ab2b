"""N>1 path of bench.py on CPU: world_size-2 gloo ranks, each with its own camera stream, the
job time is the max over ranks and the frame count is the sum (weak scaling, no data-path
collective)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    s = bench.stream_of_rank(rank)
    img = synth.frame(64, 48, t=0, stream=s)
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
    assert [r[2] for r in res] == [0, 1]              # one stream per rank
    assert res[0][3] != res[1][3]                     # independent inputs
