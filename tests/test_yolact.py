"""YOLACT protonet + post-processing: the CPU oracle pinned to the reference's
goldens (tests/golden/gen_golden_yolact.py), and the HIP path (csrc/yolact.hip, the protonet
engine) against the same.

Bars: anchors, NMS indices and the box mask are exact; box_decode / box_encode within 2 ulp-scale
(device expf / logf vs the host's vectorised exp / log); masks within 1e-6 (sigmoid of a k-term
fp32 sum); the fp32 protonet within 1e-4 of the reference (the north star's fp32 bar), fp16 / bf16
within ~3x the drift measured on MI355X (profiles/r2/parity_lowp.json)."""
import numpy as np
import pytest
import torch

from helpers import golden, record_measurement
from oracle import ref_yolact as ry
from recipe import PROTONET_CASES, protonet_case, protonet_inputs, protonet_layout

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
    cb, cn = _mask_coeffs(g)
    proto = _t(g["proto"])
    np.testing.assert_allclose(ry.assemble_mask(proto, cb, box[0, det[:24]]).numpy(), g["mask_box"],
                               rtol=0, atol=1e-6)
    np.testing.assert_allclose(ry.assemble_mask(proto, cn, None).numpy(), g["mask_nobox"], rtol=0, atol=1e-6)


def _mask_coeffs(g):
    """Coefficient rows of the stored masks (the first 24 / 5 kept detections)."""
    if "coeff_box" in g:
        return _t(g["coeff_box"]), _t(g["coeff_nobox"])
    det = _t(g["mask_det"])
    coeff = _t(g["coeff"])
    return coeff[0, det[:24]], coeff[0, det[:5]]


def _nms_keys(g):
    return [tuple(float(v) if "." in v else int(v) for v in k.split("_")[1:]) for k in g if k.startswith("nms_")]


def test_oracle_large_and_degenerate_nms_match_reference():
    g = golden("yolact_640x360_ar3")
    assert int(g["A"]) == 14505  # evaluate.py:17-34: 4835 cells x 3 aspect ratios
    for k, iou, conf in _nms_keys(g):
        np.testing.assert_array_equal(ry.nms(_t(g["cls"]), _t(g["box"]), k, iou, conf).numpy(),
                                      g[f"nms_{k}_{iou}_{conf}"])
    d = golden("yolact_degenerate")
    for k, iou, conf in _nms_keys(d):
        np.testing.assert_array_equal(ry.nms(_t(d["cls"]), _t(d["box"]), k, iou, conf).numpy(),
                                      d[f"nms_{k}_{iou}_{conf}"])


def test_oracle_box_encode_matches_reference():
    g = golden("yolact_640x360_ar3")
    enc = ry.box_encode(_t(g["gt_box"]), _t(g["anchor"]), VAR)
    np.testing.assert_allclose(enc.numpy(), g["gt_enc"], rtol=4e-7, atol=1e-7)


@pytest.mark.parametrize("name", [c["name"] for c in PROTONET_CASES])
def test_oracle_protonet_matches_reference(name):
    c, g = protonet_case(name), golden(name)
    sd, x = protonet_inputs(c)
    with torch.no_grad():
        y = ry.masknet(sd, x)
    assert tuple(y.shape) == tuple(g["out_shape"])
    if c["full"]:
        np.testing.assert_array_equal(y.numpy(), g["out"])
    else:
        np.testing.assert_array_equal(y.reshape(-1)[_t(g["sample_index"])].numpy(), g["sample"])
    np.testing.assert_allclose(y.double().sum(dim=(0, 2, 3)).numpy(), g["chan_sum"], rtol=1e-9)


def test_masknet_layout_matches_reference():
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    for F, k in ((256, 8), (32, 32), (64, 16)):
        m = Masknet(YolactConfig(640, 360, SCALES, (1,), VAR, feature_depth=F, n_prototype_masks=k))
        assert [(n, tuple(v.shape)) for n, v in m.state_dict().items()] == protonet_layout(F, k)


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
    cb, cn = (c.cuda() for c in _mask_coeffs(g))
    proto = _t(g["proto"]).cuda()
    rb = _t(ref_box).cuda()
    m = assemble_mask(proto, cb, rb[0, det[:24]]).cpu().numpy()
    np.testing.assert_allclose(m, g["mask_box"], rtol=0, atol=1e-6)
    assert ((m == 0) == (g["mask_box"] == 0)).all()  # the inclusive box mask is exact
    np.testing.assert_allclose(assemble_mask(proto, cn, None).cpu().numpy(), g["mask_nobox"], rtol=0, atol=1e-6)
    # the same prototypes read through an NHWC view (Masknet's output layout)
    nhwc = proto.permute(1, 2, 0).contiguous().permute(2, 0, 1)
    np.testing.assert_array_equal(assemble_mask(nhwc, cb, rb[0, det[:24]]).cpu().numpy(), m)


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
    # more anchors than one workgroup's LDS holds (the reference has no limit)
    g = torch.Generator().manual_seed(5)
    cls9, box9 = torch.randn(1, 30000, 3, generator=g), torch.rand(1, 30000, 4, generator=g) * 0.3
    np.testing.assert_array_equal(nms(cls9.cuda(), box9.cuda(), 300, 0.5, 0.1).cpu().numpy(),
                                  ry.nms(cls9, box9, 300, 0.5, 0.1).numpy())


@pytest.mark.gpu
def test_gpu_large_and_degenerate_nms():
    from tauv_vision_amd.yolact import nms, BatchedNMS
    for name in ("yolact_640x360_ar3", "yolact_degenerate"):
        g = golden(name)
        cls, box = _t(g["cls"]).cuda(), _t(g["box"]).cuda()
        for k, iou, conf in _nms_keys(g):
            np.testing.assert_array_equal(nms(cls, box, k, iou, conf).cpu().numpy(), g[f"nms_{k}_{iou}_{conf}"])
    # batched: every image of a batch == the reference nms of that image alone
    g = golden("yolact_550x550")
    cls, box = _t(g["cls"]), _t(g["box"])
    bn = BatchedNMS(cls.shape[0], cls.shape[1], 100, "cuda")
    det, cnt = bn(cls.cuda(), box.cuda(), 0.5, 0.05)
    det, cnt = det.cpu().numpy(), cnt.cpu().numpy()
    for b in range(cls.shape[0]):
        ref = ry.nms(cls[b:b + 1], box[b:b + 1], 100, 0.5, 0.05).numpy()
        assert cnt[b] == len(ref)
        np.testing.assert_array_equal(det[b, :cnt[b]], ref)
    # the node's mask step straight from the batched NMS output (yolact_node.py:134)
    from tauv_vision_amd.yolact import assemble_mask, assemble_masks_indexed
    gg = torch.Generator().manual_seed(11)
    B, A = cls.shape[:2]
    proto = torch.randn(B, 40, 44, 8, generator=gg).cuda().permute(0, 3, 1, 2)
    coeff = torch.randn(B, A, 8, generator=gg).cuda()
    bd, bc = bn(cls.cuda(), box.cuda(), 0.5, 0.05)
    masks = assemble_masks_indexed(proto, coeff, box.cuda(), bd, bc).cpu()
    for b in range(B):
        d = torch.from_numpy(det[b, :cnt[b]]).cuda()
        np.testing.assert_array_equal(masks[b, :cnt[b]].numpy(),
                                      assemble_mask(proto[b], coeff[b, d], box.cuda()[b, d]).cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("A", [20000, 40000])
def test_gpu_nms_streaming_sort(A):
    """nms_sort (top_k > 1024 or > 32768 anchors, up to the full sort in rank ranges of 16384)
    against the oracle. The anchors' confidences are spaced >= 10 ulps apart (a permuted ramp of
    the class-1 logit): nms_keys' softmax may differ from torch's CPU one by an ulp, which would
    swap two confidences 1 ulp apart, and the order of exactly equal ones is torch's unstable
    CPU sort order, which the reference does not define either."""
    from tauv_vision_amd.yolact import nms
    g = torch.Generator().manual_seed(A)
    logits = torch.full((1, A, 4), -10.0)
    logits[0, :, 0] = 0.0
    logits[0, :, 1] = torch.linspace(-5.0, 5.0, A)[torch.randperm(A, generator=g)]
    xy = torch.rand(1, A, 2, generator=g)
    box = torch.cat([xy, 0.02 + 0.1 * torch.rand(1, A, 2, generator=g)], -1)
    # (> 32768 anchors: the streaming kernel even at top_k 100; top_k 17000 > 16384: two rank ranges)
    cases = ((100, 0.5, 0.05), (3000, 0.5, 0.05), (A, 0.7, 0.0)) if A < 32768 else ((100, 0.5, 0.05), (17000, 0.7, 0.0))
    for k, iou, conf in cases:
        ref = ry.nms(logits, box, k, iou, conf).numpy()
        np.testing.assert_array_equal(nms(logits.cuda(), box.cuda(), k, iou, conf).cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_box_encode_matches_reference():
    from tauv_vision_amd.yolact import YolactConfig, box_encode, box_decode
    g = golden("yolact_640x360_ar3")
    cfg = YolactConfig(640, 360, SCALES, (0.5, 1, 2), VAR)
    anchor = _t(g["anchor"]).cuda()
    enc = box_encode(_t(g["gt_box"]).cuda(), anchor, cfg)
    np.testing.assert_allclose(enc.cpu().numpy(), g["gt_enc"], rtol=4e-7, atol=2e-7)
    # decode(encode(box)) == box (the round trip of boxes.py:106-117)
    np.testing.assert_allclose(box_decode(enc, anchor, cfg).cpu().numpy(), g["gt_box"], rtol=2e-6, atol=2e-7)


@pytest.mark.gpu
def test_gpu_assemble_masks_batched():
    from tauv_vision_amd.yolact import assemble_mask, assemble_masks
    g = torch.Generator().manual_seed(9)
    B, K, H, W, n = 3, 8, 37, 53, 11
    proto = torch.randn(B, H, W, K, generator=g).cuda().permute(0, 3, 1, 2)  # NHWC storage
    coeff = torch.randn(B, n, K, generator=g).cuda()
    box = torch.cat([torch.rand(B, n, 2, generator=g), torch.rand(B, n, 2, generator=g) * 0.6], -1).cuda()
    counts = torch.tensor([11, 0, 5], dtype=torch.int32).cuda()
    out = assemble_masks(proto, coeff, box, counts, out=torch.full((B, n, H, W), -1.0).cuda()).cpu()
    for b in range(B):
        c = int(counts[b])
        if c:
            np.testing.assert_array_equal(out[b, :c].numpy(), assemble_mask(proto[b], coeff[b, :c], box[b, :c]).cpu().numpy())
            ref = ry.assemble_mask(proto[b].cpu(), coeff[b, :c].cpu(), box[b, :c].cpu()).numpy()
            np.testing.assert_allclose(out[b, :c].numpy(), ref, rtol=0, atol=1e-6)
        assert (out[b, c:] == -1.0).all()  # rows past the count untouched


@pytest.mark.gpu
@pytest.mark.parametrize("K", [3, 8, 12, 16, 20, 37])
@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
def test_gpu_assemble_mask_prototype_counts(K, layout):
    """Both mask kernels (prototypes in registers for K <= 16 in two widths, LDS-staged above),
    NCHW and NHWC prototype storage, a width not a multiple of 4 (scalar stores) and one that is."""
    from tauv_vision_amd.yolact import assemble_mask
    g = torch.Generator().manual_seed(K)
    for H, W in ((19, 23), (16, 36)):
        p = torch.randn(K, H, W, generator=g)
        proto = p.cuda() if layout == "nchw" else p.permute(1, 2, 0).contiguous().cuda().permute(2, 0, 1)
        n = 70  # two detection chunks of the kernels
        coeff = torch.randn(n, K, generator=g)
        box = torch.cat([torch.rand(n, 2, generator=g), torch.rand(n, 2, generator=g) * 0.6], -1)
        for bx in (box, None):
            got = assemble_mask(proto, coeff.cuda(), None if bx is None else bx.cuda()).cpu().numpy()
            ref = ry.assemble_mask(p, coeff, bx).numpy()
            np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_gpu_assemble_masks_rejects_bad_out():
    """A caller-supplied `out` / index tensor reaches the kernel as a raw pointer: wrong shape,
    dtype, layout or device is refused before any launch (nothing is written)."""
    from tauv_vision_amd.yolact import assemble_masks, assemble_masks_indexed
    B, K, H, W, n, A = 2, 8, 9, 13, 3, 20
    proto = torch.randn(B, K, H, W).cuda()
    coeff = torch.randn(B, n, K).cuda()
    for bad in (torch.empty(B, n, H, W + 1).cuda(), torch.empty(B, n, H, W, dtype=torch.float16).cuda(),
                torch.empty(B, n, W, H).cuda().transpose(2, 3), torch.empty(B, n, H, W)):
        with pytest.raises(ValueError):
            assemble_masks(proto, coeff, None, out=bad)
    with pytest.raises(ValueError):
        assemble_masks(proto, coeff, None, counts=torch.zeros(B, dtype=torch.int32))  # host counts
    acoeff = torch.randn(B, A, K).cuda()
    det = torch.zeros(B, n, dtype=torch.int64).cuda()
    cnt = torch.ones(B, dtype=torch.int32).cuda()
    with pytest.raises(ValueError):
        assemble_masks_indexed(proto, acoeff, None, det.cpu(), cnt)
    with pytest.raises(ValueError):
        assemble_masks_indexed(proto, acoeff, None, det, cnt, out=torch.empty(B, n + 1, H, W).cuda())
    good = assemble_masks_indexed(proto, acoeff, None, det, cnt, out=torch.empty(B, n, H, W).cuda())
    assert good.shape == (B, n, H, W)


PROTO_TOL = {"fp32": 1e-4, "fp32x3": 1e-4, "fp16": 8e-4, "bf16": 6e-3}  # ~3x the MI355X drift (profiles/r2/parity_yolact.json)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp32x3", "fp16", "bf16"])
@pytest.mark.parametrize("name", [c["name"] for c in PROTONET_CASES])
def test_gpu_protonet_matches_reference(name, precision):
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    c, g = protonet_case(name), golden(name)
    sd, x = protonet_inputs(c)
    m = Masknet(YolactConfig(640, 360, SCALES, (1,), VAR, feature_depth=c["F"], n_prototype_masks=c["k"]),
                precision=precision)
    m.load_state_dict(sd)
    y = m(x.cuda())
    assert tuple(y.shape) == tuple(g["out_shape"])
    y = y.cpu()
    if c["full"]:
        err = float(np.abs(y.numpy() - g["out"]).max())
        scale = float(np.abs(g["out"]).max())
    else:
        got = y.reshape(-1)[_t(g["sample_index"])].numpy() if y.is_contiguous() else \
            y.contiguous().reshape(-1)[_t(g["sample_index"])].numpy()
        err = float(np.abs(got - g["sample"]).max())
        scale = float(np.abs(g["sample"]).max())
    record_measurement(f"protonet/{name}/{precision}", {"max_abs_err": err, "ref_absmax": scale})
    assert err <= PROTO_TOL[precision] * max(1.0, scale), f"{name} {precision}: {err}"
    # per-channel sums over every output (not just the sample): independent per-element errors
    # grow like sqrt(n); a systematic bias would grow like n and fail this
    npix = y.shape[0] * y.shape[2] * y.shape[3]
    np.testing.assert_allclose(y.double().sum(dim=(0, 2, 3)).numpy(), g["chan_sum"], rtol=PROTO_TOL[precision],
                               atol=4 * PROTO_TOL[precision] * max(1.0, scale) * npix ** 0.5)


@pytest.mark.gpu
def test_gpu_protonet_batch_consistency():
    """Frames are independent: a batch (incl. the two concurrent slices of B >= 16) gives every
    frame its single-frame result — within fp16 rounding, since the kernel choice may depend on
    the batch (the split-K conv_lat for layers a small batch leaves under-filled sums K in
    another order) — and a repeated run of the same batch is bit-identical."""
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    c = protonet_case("protonet_f64_k16_b1_9x17")
    sd, _ = protonet_inputs(c)
    m = Masknet(YolactConfig(640, 360, SCALES, (1,), VAR, feature_depth=64, n_prototype_masks=16), precision="fp16")
    m.load_state_dict(sd)
    x = torch.randn(17, 64, 9, 17, generator=torch.Generator().manual_seed(4)).cuda()
    yb = m(x).cpu()
    np.testing.assert_array_equal(m(x).cpu().numpy(), yb.numpy())
    scale = max(1.0, float(yb.abs().max()))
    for i in (0, 8, 16):
        np.testing.assert_allclose(m(x[i:i + 1]).cpu().numpy(), yb[i:i + 1].numpy(), rtol=0, atol=1e-3 * scale)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_gpu_protonet_bench_batch_matches_reference(precision):
    """The protonet bench.py --model yolact times (BASELINE config 5: F = 256 at the 550x550 fpn[0]
    of 69x69, batch 32 = two concurrent 16-frame slices, the 256-channel halo convs and the
    full-size ConvTranspose phase GEMMs of that batch) on the reference's golden input placed at the
    first frame of each slice: output samples and per-channel sums against the reference Masknet's
    (masknet.py:45-55; the bench line's `parity` leg runs this same function)."""
    import bench
    res = bench.yolact_parity(32, precision, torch.device("cuda", 0))
    record_measurement(f"protonet/f256_69x69_b32/{precision}", res)
    assert res["slices"] == [16, 16], res
    assert res["frames_checked"] == 2, res
    assert res["within_tol"], res
