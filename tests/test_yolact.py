"""YOLACT post-processing: the CPU oracle pinned to the reference's goldens
(tests/golden/gen_golden_yolact.py), and the HIP kernels (csrc/yolact.hip) against the same.

Bars: anchors, NMS indices and the box mask are exact; box_decode within 2 ulp-scale (device
expf vs the host's vectorised exp); masks within 1e-6 (sigmoid of an 8-term fp32 sum)."""
import numpy as np
import pytest
import torch

from helpers import golden
from oracle import ref_yolact as ry

CASES = {
    "yolact_640x360": dict(in_w=640, in_h=360, fpn=[(45, 80), (23, 40), (12, 20), (6, 10), (3, 5)], ars=(1,)),
    "yolact_550x550": dict(in_w=550, in_h=550, fpn=[(69, 69), (35, 35), (18, 18), (9, 9), (5, 5)], ars=(1,)),
    "yolact_256x256_ar3": dict(in_w=256, in_h=256, fpn=[(32, 32), (16, 16), (8, 8), (4, 4), (2, 2)],
                               ars=(1, 0.5, 2)),
}
SCALES, VAR = (24, 48, 96, 192, 384), (0.1, 0.2)
NMS_KEYS = [(100, 0.5, 0.05), (200, 0.3, 0.2), (50, 0.7, 0.0)]


def _t(a):
    return torch.from_numpy(np.asarray(a))


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_matches_reference(name):
    c, g = CASES[name], golden(name)
    anchor = torch.cat([ry.get_anchor(i, s, SCALES, c["ars"], c["in_h"], c["in_w"]) for i, s in enumerate(c["fpn"])], 1)
    np.testing.assert_array_equal(anchor.numpy(), g["anchor"])
    box = ry.box_decode(_t(g["enc"]), anchor, VAR)
    # torch.exp is vectorised per host ISA: bit-exact on the golden host, ulp-close elsewhere
    np.testing.assert_allclose(box.numpy(), g["box"], rtol=4e-7, atol=0)
    box = _t(g["box"])
    for k, iou, conf in NMS_KEYS:
        np.testing.assert_array_equal(ry.nms(_t(g["cls"]), box, k, iou, conf).numpy(), g[f"nms_{k}_{iou}_{conf}"])
    det = _t(g["mask_det"])
    coeff, proto = _t(g["coeff"]), _t(g["proto"])
    np.testing.assert_allclose(ry.assemble_mask(proto, coeff[0, det[:24]], box[0, det[:24]]).numpy(), g["mask_box"],
                               rtol=0, atol=1e-6)
    np.testing.assert_allclose(ry.assemble_mask(proto, coeff[0, det[:5]], None).numpy(), g["mask_nobox"], rtol=0,
                               atol=1e-6)


def test_drop_in_get_anchor_matches_reference():
    from tauv_vision_amd.yolact import YolactConfig, get_anchor
    for name, c in CASES.items():
        cfg = YolactConfig(c["in_w"], c["in_h"], SCALES, c["ars"], VAR)
        anchor = torch.cat([get_anchor(i, s, cfg) for i, s in enumerate(c["fpn"])], 1)
        np.testing.assert_array_equal(anchor.numpy(), golden(name)["anchor"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_postprocess_matches_reference(name):
    from tauv_vision_amd.yolact import YolactConfig, box_decode, nms, assemble_mask
    c, g = CASES[name], golden(name)
    cfg = YolactConfig(c["in_w"], c["in_h"], SCALES, c["ars"], VAR)
    anchor = _t(g["anchor"]).cuda()
    box = box_decode(_t(g["enc"]).cuda(), anchor, cfg)
    ref_box = g["box"]
    np.testing.assert_allclose(box.cpu().numpy(), ref_box, rtol=4e-7, atol=1e-7)
    # NMS on the reference's boxes (so the indices test NMS alone) and on ours
    cls = _t(g["cls"]).cuda()
    for k, iou, conf in NMS_KEYS:
        ref = g[f"nms_{k}_{iou}_{conf}"]
        np.testing.assert_array_equal(nms(cls, _t(ref_box).cuda(), k, iou, conf).cpu().numpy(), ref)
        np.testing.assert_array_equal(nms(cls, box, k, iou, conf).cpu().numpy(), ref)
    det = _t(g["mask_det"])
    coeff, proto = _t(g["coeff"]).cuda(), _t(g["proto"]).cuda()
    rb = _t(ref_box).cuda()
    m = assemble_mask(proto, coeff[0, det[:24]], rb[0, det[:24]]).cpu().numpy()
    np.testing.assert_allclose(m, g["mask_box"], rtol=0, atol=1e-6)
    assert ((m == 0) == (g["mask_box"] == 0)).all()  # the inclusive box mask is exact
    np.testing.assert_allclose(assemble_mask(proto, coeff[0, det[:5]], None).cpu().numpy(), g["mask_nobox"], rtol=0,
                               atol=1e-6)


@pytest.mark.gpu
def test_gpu_postprocess_edge_cases():
    from tauv_vision_amd.yolact import nms, assemble_mask
    # nothing passes the confidence threshold -> empty result (the node's `len(detections) == 0`)
    cls = torch.zeros(1, 10, 3).cuda()
    box = torch.rand(1, 10, 4).cuda()
    assert nms(cls, box, 5, 0.5, 0.99).numel() == 0
    # top_k larger than the anchor count; a single anchor
    assert nms(torch.randn(1, 1, 3).cuda(), box[:, :1], 100, 0.5, 0.0).tolist() == [0]
    # zero detections -> [0, H, W]
    assert assemble_mask(torch.rand(4, 8, 8).cuda(), torch.zeros(0, 4).cuda(), None).shape == (0, 8, 8)
    with pytest.raises(RuntimeError):  # the one-workgroup kernel's documented limit (8192 anchors)
        nms(torch.randn(1, 9000, 3).cuda(), torch.rand(1, 9000, 4).cuda(), 10, 0.5, 0.1)
