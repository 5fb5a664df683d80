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
        buf = g(RecordGather.pack(rec, cnt))  # one collective: records + counts in one buffer
        assert buf.shape == (world, (per * K * REC + per) * 4)
        all_rec, all_cnt = g.unpack()
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


# ---- end to end: per-rank forward + decode of a frame shard -> RecordGather -> detections ----
E2E = dict(heights=[2] * 5, channels=[16] * 6, ds=2, H=96, W=128, K=20, thr=0.05, n=5)


def _e2e_frames():
    from recipe import seeded_u8_frames, normalize
    fr = seeded_u8_frames(E2E["n"], E2E["H"], E2E["W"], seed=21)
    return normalize(fr.permute(0, 3, 1, 2).float() / 255.0)


def _e2e_sd():
    import oracle
    from recipe import seeded_state_dict
    from tauv_vision_amd.weights import model_desc, param_layout
    desc = model_desc(E2E["heights"], E2E["channels"], E2E["ds"], [4, 2, 2])
    return seeded_state_dict(param_layout(desc)), oracle


def _pack(dets, K):
    """One frame's decode() output in the device record layout [K, 10] + count (decode.hip
    merge_select: label, score, y, x, h, w, depth, flat index, aux0, aux1)."""
    r = np.zeros((K, REC), np.float32)
    for i, (lab, sc, y, x, h, w, d) in enumerate(dets):
        r[i, :7] = (lab, sc, y, x, h, w, np.nan if d is None else d)
    return r, len(dets)


def e2e_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sd, oracle = _e2e_sd()
        img = _e2e_frames()
        n, K = E2E["n"], E2E["K"]
        lo, hi = shard_bounds(n, rank, world)
        per = -(-n // world)
        rec = torch.zeros((per, K, REC))
        cnt = torch.zeros((per,), dtype=torch.int32)  # short shard: padded frames with 0 records
        if hi > lo:
            with torch.no_grad():
                pred = oracle.centernet_forward(sd, img[lo:hi], E2E["heights"], E2E["ds"], {})
            for i, dets in enumerate(oracle.decode(pred, E2E["H"], E2E["W"], E2E["ds"], K, E2E["thr"])):
                r, c = _pack(dets, K)
                rec[i], cnt[i] = torch.from_numpy(r), c
        g = RecordGather(per, K, "cpu")
        g(RecordGather.pack(rec, cnt))
        all_rec, all_cnt = g.unpack()
        if rank == 0:
            q.put((all_rec[:n].numpy().copy(), all_cnt[:n].numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_sharded_forward_decode_gather_matches_single_process():
    """Frames sharded over 2 gloo ranks (5 frames: shards of 3 and 2), each rank runs forward +
    decode on its own frames, one all-gather of the fixed-size records, host conversion — equals
    decode() of the whole batch in one process (frames are independent)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=e2e_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rec, cnt = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd, oracle = _e2e_sd()
    with torch.no_grad():
        pred = oracle.centernet_forward(sd, _e2e_frames(), E2E["heights"], E2E["ds"], {})
    want = oracle.decode(pred, E2E["H"], E2E["W"], E2E["ds"], E2E["K"], E2E["thr"])
    got = records_to_detections(rec, cnt, has_depth=False)
    assert [len(g) for g in got] == [len(w) for w in want]
    for gb, wb in zip(got, want):
        for d, w in zip(gb, wb):
            assert int(d.label) == w[0]
            assert float(d.score) == np.float32(w[1])
            assert d.y == float(np.float32(w[2])) and d.x == float(np.float32(w[3]))
            assert d.h == w[4] and d.w == w[5]
