"""Multi-process (gloo, world_size 2, CPU) coverage of the frame-sharded path: shard bounds,
the records all-gather (RecordGather, the bench's only collective) and the host conversion of
gathered records into decode()'s List[List[Detection]]."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tauv_vision_amd.decode import REC
from tauv_vision_amd.sharding import RecordGather, records_to_detections, shard_bounds

K = 5


def frame_records(f):
    """Deterministic stand-in for one frame's device records and count."""
    r = np.zeros((K, REC), np.float32)
    r[:, 0] = np.arange(K) % 3
    r[:, 1] = 1.0 - 0.1 * np.arange(K) - 0.001 * f
    r[:, 2:6] = f + np.arange(4)[None, :] * 0.25
    r[:, 6] = 2.0 + f
    r[:, 7] = np.arange(K) + 100 * f
    return r, f % (K + 1)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, n, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(n, rank, world)
        per = -(-n // world)
        rec = torch.zeros((per, K, REC))
        cnt = torch.zeros((per,), dtype=torch.int32)
        for i, f in enumerate(range(lo, hi)):
            r, c = frame_records(f)
            rec[i] = torch.from_numpy(r)
            cnt[i] = c
        g = RecordGather(per, K, "cpu")
        all_rec, all_cnt = g(rec, cnt)
        if rank == 0:
            q.put((all_rec[:n].numpy().copy(), all_cnt[:n].numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [8, 7])
def test_record_gather_two_ranks(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    rec, cnt = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for f in range(n):
        r, c = frame_records(f)
        assert np.array_equal(rec[f], r)
        assert cnt[f] == c
    dets = records_to_detections(rec, cnt, has_depth=True)
    assert [len(d) for d in dets] == [f % (K + 1) for f in range(n)]
    d = dets[3][1]
    r, _ = frame_records(3)
    assert int(d.label) == int(r[1, 0]) and d.y == float(r[1, 2]) and d.depth == float(r[1, 6])


def test_shard_bounds():
    assert [shard_bounds(10, r, 4) for r in range(4)] == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert [shard_bounds(2, r, 4) for r in range(4)] == [(0, 1), (1, 2), (2, 2), (2, 2)]
    assert shard_bounds(64, 0, 1) == (0, 64)
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)
