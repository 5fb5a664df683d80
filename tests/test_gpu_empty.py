"""Empty batches through the drop-in API, with the reference's own semantics (checked against the
oracle restatement, which runs the reference's torch ops on the CPU):

  * a forward of B = 0 frames returns empty Prediction tensors of the usual per-frame shapes (the
    reference's convolutions accept an empty batch) — R18, DLA-34, the standalone backbone, the
    protonet, and forward_frames / preprocess;
  * heatmap_nms returns the empty batch (decode.py:239-252: max_pool2d);
  * heatmap_detect, decode and decode_keypoints raise RuntimeError, as the reference's
    heatmap_detect does (decode.py:255-279: `reshape(B, -1)` of 0 elements).
"""
import pytest
import torch

from helpers import case_by_name

import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu

NAME = "r18_c128_b1_480x640"


def test_empty_heatmap_ops_match_reference():
    from oracle import ref_decode as rd
    import tauv_vision_amd as tv
    h = torch.zeros((0, 4, 120, 160))
    assert tuple(tv.heatmap_nms(h.cuda(), 3).shape) == tuple(rd.heatmap_nms(h, 3).shape)
    with pytest.raises(RuntimeError):
        rd.heatmap_detect(h, 100)
    with pytest.raises(RuntimeError):
        tv.heatmap_detect(h.cuda(), 100)


@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_empty_forward_r18(precision):
    import tauv_vision_amd as tv
    model, oc, mc, case = fwd.build(NAME, precision)
    H, W = case["in_h"], case["in_w"]
    one = model(torch.zeros((1, 3, H, W), device="cuda"))
    for pred in (model(torch.zeros((0, 3, H, W), device="cuda")),
                 model.forward_frames(torch.zeros((0, H, W, 3), dtype=torch.uint8, device="cuda")),
                 model.forward_frames(torch.zeros((0, 2 * H, 2 * W, 3), dtype=torch.uint8, device="cuda"), (H, W))):
        for f in ("heatmap", "size", "offset"):
            got, ref = getattr(pred, f), getattr(one, f)
            assert tuple(got.shape) == (0,) + tuple(ref.shape[1:]), f
    empty = model(torch.zeros((0, 3, H, W), device="cuda"))
    with pytest.raises(RuntimeError):
        tv.decode(empty, mc, 100, 0.3)
    # the engine still runs a real batch afterwards
    again = model(torch.zeros((1, 3, H, W), device="cuda"))
    assert torch.equal(again.heatmap, one.heatmap)


def test_empty_forward_backbone_dla34_protonet():
    import tauv_vision_amd as tv
    case = case_by_name(NAME)
    bb = tv.DLABackbone(case["heights"], case["channels"], case["downsamples"]).cuda().eval()
    H, W = case["in_h"], case["in_w"]
    ref = bb(torch.zeros((1, 3, H, W), device="cuda"))
    got = bb(torch.zeros((0, 3, H, W), device="cuda"))
    assert tuple(got.shape) == (0,) + tuple(ref.shape[1:])
    A = tv.AngleConfig
    oc = tv.ObjectConfigSet([tv.ObjectConfig("o0", A(False, 1.0), A(False, 1.0), A(False, 1.0), False, True,
                                             [(0.0, 0.0, 0.0)])])
    dla = tv.CenterpointDLA34(oc, precision="fp16").cuda().eval()
    p1 = dla(torch.zeros((1, 3, 256, 320), device="cuda"))
    p0 = dla(torch.zeros((0, 3, 256, 320), device="cuda"))
    for f in ("heatmap", "keypoint_heatmap", "keypoint_affinity", "size"):
        assert tuple(getattr(p0, f).shape) == (0,) + tuple(getattr(p1, f).shape[1:]), f
    with pytest.raises(RuntimeError):
        tv.decode_keypoints(p0, tv.ModelConfig([], [], 256, 320, 2, 1.0), oc, None, 10, 10, 0.3, 0.3, 0.0)
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    net = Masknet(YolactConfig(550, 550, (24, 48, 96, 192, 384), (1,), (0.1, 0.2), feature_depth=64,
                               n_prototype_masks=8), precision="fp16").cuda()
    y1 = net(torch.zeros((1, 64, 35, 35), device="cuda"))
    y0 = net(torch.zeros((0, 64, 35, 35), device="cuda"))
    assert tuple(y0.shape) == (0,) + tuple(y1.shape[1:])
