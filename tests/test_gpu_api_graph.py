"""The drop-in API's hipGraph cache (centernet.py _NativeModel._launch): the reference-shaped calls
`model(img)` / `model.forward_frames(frames)` run eagerly the first time a (kind, shape) is seen,
capture the forward once on the second call and replay it from then on. Checked here, against the
same model with graph_replay off (every launch eager):

  * every replayed call returns the eager heads bit for bit, for new inputs each call (the static
    input buffer is refreshed, nothing is served from the capture);
  * returned tensors are fresh: a later call does not change an earlier call's Prediction;
  * the node's per-frame sequence (centernet_node.py:94,106-116: CenterpointDLA34 forward of a
    normalised fp32 image, then decode_keypoints with K=10/50, thr 0.6/0.3) gives the same
    detections replayed as eager, in the drop-in default fp32 and in fp16;
  * decode_records (cached decoder, one D2H) equals decode()'s detections.
"""
import numpy as np
import pytest
import torch

import bench

pytestmark = pytest.mark.gpu


def _heads(pred):
    return torch.cat([pred.heatmap.permute(0, 2, 3, 1).reshape(-1), pred.size.reshape(-1),
                      pred.offset.reshape(-1)])


@pytest.mark.parametrize("arch,precision,B", [("r18", "fp32", 1), ("r18", "fp16", 1), ("r18", "bf16", 3),
                                              ("dla34", "fp16", 1)])
def test_forward_replay_matches_eager(arch, precision, B):
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model(precision, dev, arch)
    ref, _, _ = bench.build_model(precision, dev, arch)
    ref.graph_replay = False
    outs = []
    for i in range(4):
        img = torch.randn((B, 3, 480, 640), generator=torch.Generator().manual_seed(40 + i)).to(dev)
        got = model(img)
        want = ref(img)
        torch.cuda.synchronize()
        assert torch.equal(_heads(got), _heads(want)), f"call {i}"
        outs.append((got, _heads(got).clone()))
    assert any(e.get("graph") is not None for e in model._graphs.values()), "no graph captured"
    assert getattr(model, "graph_failures", 0) == 0
    for got, snap in outs:  # fresh outputs: later calls left them untouched
        assert torch.equal(_heads(got), snap)


def test_forward_frames_replay_matches_eager():
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model("fp16", dev, "r18")
    ref, _, _ = bench.build_model("fp16", dev, "r18")
    ref.graph_replay = False
    for i in range(3):
        frames = torch.randint(0, 256, (2, 480, 640, 3), generator=torch.Generator().manual_seed(60 + i),
                               dtype=torch.uint8).to(dev)
        assert torch.equal(_heads(model.forward_frames(frames)), _heads(ref.forward_frames(frames)))
    assert any(e.get("graph") is not None for e in model._graphs.values())


@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_node_sequence_replay_matches_eager(precision):
    from tauv_vision_amd.decode import decode_keypoints
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model(precision, dev, "dla34")
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
    M = np.array([[307.0, 0.0, 160.0], [0.0, 307.0, 120.0], [0.0, 0.0, 0.0]])
    img = torch.randn((1, 3, 480, 640), generator=torch.Generator().manual_seed(9)).to(dev)
    model(img)  # the node's warm-up forward (centernet_node.py:50)
    runs = []
    for replay in (True, True, False):
        model.graph_replay = replay
        dets = decode_keypoints(model(img), mc, oc, M, 10, 50, 0.6, 0.3, 0.3)[0]
        runs.append([(d.label, d.score, d.y, d.x, d.h, d.w, d.depth, tuple(map(str, d.keypoints))) for d in dets])
    assert runs[0] == runs[1] == runs[2]


def test_decode_records_matches_decode():
    from tauv_vision_amd.decode import decode, decode_records
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model("fp16", dev, "r18")
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
    frames = torch.randint(0, 256, (3, 480, 640, 3), generator=torch.Generator().manual_seed(2),
                           dtype=torch.uint8).to(dev)
    pred = model.forward_frames(frames)
    for _ in range(2):  # the second call reuses the cached decoder and its workspace
        rec, cnt = decode_records(pred, mc, 100, 0.3)
        dets = decode(pred, mc, 100, 0.3)
        assert [len(d) for d in dets] == cnt.tolist()
        for b, db in enumerate(dets):
            for i, d in enumerate(db):
                assert int(d.label) == int(rec[b, i, 0]) and float(d.score) == float(rec[b, i, 1])
                assert (d.y, d.x, d.h, d.w) == tuple(float(v) for v in rec[b, i, 2:6])
