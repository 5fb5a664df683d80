"""GPU parity of the decode kernels (peak NMS, exact top-K, records) against the
reference's golden vectors and the CPU oracle. Bit-exact indices; fp32 values."""
import numpy as np
import pytest
import torch

import oracle
from helpers import golden
from recipe import decode_case_inputs, gaussian_blob

pytestmark = pytest.mark.gpu

CASES = ["decode_b3_c4_120x160", "decode_b2_c4_90x160", "decode_b1_c80_64x64"]


def _inputs(name):
    g = golden(name)
    seed, B, C, H, W = [int(v) for v in g["seed"]]
    return g, decode_case_inputs(B, C, H, W, seed)


@pytest.mark.parametrize("name", CASES)
def test_nms_and_topk_match_golden(name):
    from tauv_vision_amd import heatmap_nms, heatmap_detect
    g, (logits, size, offset, depth) = _inputs(name)
    sig = torch.sigmoid(logits).cuda()
    nms = heatmap_nms(sig, 3)
    # peak set bit-exact; values are the input values (no arithmetic)
    np.testing.assert_array_equal(nms.cpu().numpy(), g["nms"])
    idx, lab, score = heatmap_detect(nms, 100)
    np.testing.assert_array_equal(idx.cpu().numpy(), g["index"])
    np.testing.assert_array_equal(lab.cpu().numpy(), g["label"])
    np.testing.assert_array_equal(score.cpu().numpy(), g["score"])
    assert idx.dtype == torch.int64 and lab.dtype == torch.int64 and score.dtype == torch.float32


class _P:
    pass


def _check(got, ref, has_depth, tol=1e-5):
    B = ref.shape[0]
    for b in range(B):
        n_ref = int(np.nansum(ref[b, :, 7]))
        assert len(got[b]) == n_ref, (b, len(got[b]), n_ref)
        for i, d in enumerate(got[b]):
            assert int(d.label) == int(ref[b, i, 0])
            assert isinstance(d.label, torch.Tensor) and d.label.dim() == 0
            np.testing.assert_allclose(float(d.score), ref[b, i, 1], rtol=0, atol=1e-6)
            np.testing.assert_allclose([d.y, d.x, d.h, d.w], ref[b, i, 2:6], rtol=tol, atol=tol)
            if has_depth:
                np.testing.assert_allclose(d.depth, ref[b, i, 6], rtol=1e-5, atol=1e-5)
            else:
                assert d.depth is None


@pytest.mark.parametrize("name", CASES)
def test_decode_matches_golden(name):
    import tauv_vision_amd as tv
    g, (logits, size, offset, depth) = _inputs(name)
    in_h, in_w, ds = [int(v) for v in g["meta"]]
    mc = tv.ModelConfig([], [], in_h, in_w, ds, 1.0)
    p = _P()
    p.heatmap, p.size, p.offset, p.depth = logits.cuda(), size.cuda(), offset.cuda(), depth.cuda()
    for thr in (0.05, 0.3, 0.9):
        _check(tv.decode(p, mc, 100, thr), g[f"decode_thr{thr}"], True)
    p.depth = None
    _check(tv.decode(p, mc, 100, 0.3), g["decode_nodepth_thr0.3"], False)


def test_decode_strided_nhwc_views():
    """The engine hands decode NHWC channel-slice views; results must not depend on strides."""
    import tauv_vision_amd as tv
    g, (logits, size, offset, depth) = _inputs("decode_b3_c4_120x160")
    nhwc = torch.cat([logits.permute(0, 2, 3, 1), size, offset, depth], dim=3).contiguous().cuda()
    p = _P()
    p.heatmap = nhwc[..., 0:4].permute(0, 3, 1, 2)
    p.size, p.offset, p.depth = nhwc[..., 4:6], nhwc[..., 6:8], nhwc[..., 8:9]
    mc = tv.ModelConfig([], [], 480, 640, 2, 1.0)
    _check(tv.decode(p, mc, 100, 0.3), g["decode_thr0.3"], True)


def test_kat_two_blobs():
    """decode.py:327-339 known-answer test (restated Gaussian)."""
    from tauv_vision_amd import heatmap_nms, heatmap_detect
    h = torch.cat((gaussian_blob(512, 512, 100, 100, 50)[None, None],
                   gaussian_blob(512, 512, 200, 200, 50)[None, None]), dim=1).cuda()
    idx, lab, score = heatmap_detect(heatmap_nms(h, 3), 100)
    g = golden("kat_two_blobs")
    np.testing.assert_array_equal(idx[:, :2].cpu().numpy(), g["index"])
    np.testing.assert_array_equal(lab[:, :2].cpu().numpy(), g["label"])
    np.testing.assert_array_equal(score[:, :2].cpu().numpy(), g["score"])
    assert idx[0, 0].tolist() == [100, 100]


def test_topk_edge_cases():
    from tauv_vision_amd import heatmap_detect, heatmap_nms
    # all zeros: ties everywhere -> the K smallest flat indices (deterministic tie rule)
    z = torch.zeros(2, 3, 7, 9, device="cuda")
    idx, lab, score = heatmap_detect(z, 20)
    flat = (lab * 63 + idx[..., 0] * 9 + idx[..., 1]).cpu()
    assert torch.equal(flat, torch.arange(20).repeat(2, 1))
    assert float(score.abs().sum()) == 0.0
    # K == n and K == 1 against a full sort of distinct values
    x = torch.randperm(2 * 3 * 7 * 9).float().reshape(2, 3, 7, 9).cuda()
    for K in (1, 189):
        idx, lab, score = heatmap_detect(x, K)
        ref = torch.sort(x.reshape(2, -1), dim=1, descending=True)
        np.testing.assert_array_equal(score.cpu().numpy(), ref.values[:, :K].cpu().numpy())
        flat = lab * 63 + idx[..., 0] * 9 + idx[..., 1]
        np.testing.assert_array_equal(flat.cpu().numpy(), ref.indices[:, :K].cpu().numpy())
    with pytest.raises(RuntimeError):
        heatmap_detect(x, 190)
    with pytest.raises(AssertionError):
        heatmap_nms(x, 2)
    # heavy ties: one value repeated far beyond the LDS bucket (> 4096 equal keys)
    big = torch.full((1, 4, 64, 64), 0.5, device="cuda")
    big[0, 1, 5, 7] = 0.75
    idx, lab, score = heatmap_detect(big, 300)
    assert (lab[0, 0].item(), idx[0, 0].tolist()) == (1, [5, 7])
    flat = (lab * 4096 + idx[..., 0] * 64 + idx[..., 1])[0, 1:].cpu()
    assert torch.equal(flat, torch.arange(299))
    # negative values and k=1 / k=5 windows against the oracle
    y = torch.randn(2, 3, 17, 23)
    for k in (1, 3, 5):
        np.testing.assert_array_equal(heatmap_nms(y.cuda(), k).cpu().numpy(), oracle.heatmap_nms(y, k).numpy())


def test_saturated_sigmoid_ties_are_peaks():
    """NMS compares sigmoid values: neighbours that saturate to 1.0 are all peaks (decode.py:252)."""
    import tauv_vision_amd as tv
    logits = torch.full((1, 1, 8, 8), -5.0)
    logits[0, 0, 3, 3] = 30.0
    logits[0, 0, 3, 4] = 40.0   # sigmoid(30) == sigmoid(40) == 1.0 in fp32
    ref = oracle.heatmap_nms(torch.sigmoid(logits), 3)
    got = tv.heatmap_nms(torch.sigmoid(logits).cuda(), 3).cpu()
    assert torch.equal(got, ref) and int((ref == 1.0).sum()) == 2


def _tie_rule_topk(x, K):
    """[B, n] -> (score, flat) of the top K with ties to the smaller flat index (the kernel's
    deterministic rule; torch.topk leaves tie order unspecified, decode.py:269)."""
    out_s, out_i = [], []
    for row in x:
        order = np.lexsort((np.arange(row.size), -row.astype(np.float64)))[:K]
        out_s.append(row[order])
        out_i.append(order)
    return np.stack(out_s), np.stack(out_i)


@pytest.mark.parametrize("shape,K", [((1, 4, 400, 400), 1024),   # 80 tiles > 16 per merge: two merge levels
                                     ((2, 80, 64, 64), 100),     # channel-group tiles
                                     ((3, 1, 1, 5000), 7),       # one row wider than a column band
                                     ((64, 4, 120, 160), 100)])  # the bench's decode shape
def test_topk_multi_tile_matches_sort(shape, K):
    from tauv_vision_amd import heatmap_detect, heatmap_nms
    g = torch.Generator().manual_seed(sum(shape) + K)
    x = torch.randn(shape, generator=g)
    nms = heatmap_nms(torch.sigmoid(x).cuda(), 3)
    idx, lab, score = heatmap_detect(nms, K)
    B, C, H, W = shape
    ref_s, ref_i = _tie_rule_topk(nms.cpu().numpy().reshape(B, -1), K)
    flat = (lab * H * W + idx[..., 0] * W + idx[..., 1]).cpu().numpy()
    np.testing.assert_array_equal(score.cpu().numpy(), ref_s)
    np.testing.assert_array_equal(flat, ref_i)


def test_fused_decode_matches_oracle_large_batch():
    """tv_decode (fused NMS + selection + records) at B=64 on continuous random heads vs the CPU
    oracle decode (K=100, every record: thr 0) — peak cells, scores and boxes."""
    import tauv_vision_amd as tv
    from tauv_vision_amd.decode import DeviceDecoder
    g = torch.Generator().manual_seed(77)
    B, C, H, W, K = 64, 4, 120, 160, 100
    logits = torch.randn((B, C, H, W), generator=g) * 3.0
    size = torch.randn((B, H, W, 2), generator=g) * 10.0
    offset = torch.rand((B, H, W, 2), generator=g)
    dec = DeviceDecoder(B, C, H, W, K, torch.device("cuda"))
    rec, cnt = dec(logits.cuda(), size.cuda(), offset.cuda(), None, 0, 4, 480, 640, 0.0)
    rec = rec.cpu().numpy()
    assert (cnt.cpu().numpy() == K).all()
    sig = torch.sigmoid(logits)
    nms = oracle.heatmap_nms(sig, 3).reshape(B, -1).numpy()
    ref_s, ref_i = _tie_rule_topk(nms, K)
    np.testing.assert_array_equal(rec[..., 7].astype(np.int64), ref_i)
    np.testing.assert_allclose(rec[..., 1], ref_s, rtol=0, atol=1e-6)  # device expf vs CPU sigmoid
    lab, rem = ref_i // (H * W), ref_i % (H * W)
    iy, ix = rem // W, rem % W
    bi = np.arange(B)[:, None]
    np.testing.assert_array_equal(rec[..., 0], lab)
    np.testing.assert_array_equal(rec[..., 4], size.numpy()[bi, iy, ix, 0])
    np.testing.assert_array_equal(rec[..., 5], size.numpy()[bi, iy, ix, 1])
    y = ((4.0 * iy + offset.numpy()[bi, iy, ix, 0].astype(np.float64)) / 480).astype(np.float32)
    np.testing.assert_array_equal(rec[..., 2], y)


def test_decode_fallback_and_workspace_reuse():
    """Images with fewer than K positive peaks (sigmoid saturated to 0: the exact streaming path)
    next to ordinary ones, decoded three times through one DeviceDecoder with the images rotated
    (the per-tile key segments of one call must not leak into the next)."""
    from tauv_vision_amd.decode import DeviceDecoder
    B, C, H, W, K = 3, 2, 20, 30, 50
    g = torch.Generator().manual_seed(5)
    logits = torch.full((B, C, H, W), -200.0)              # image 0: every score 0
    pos = torch.randperm(C * H * W, generator=g)[:10]      # image 1: 10 positive peaks < K
    logits[1].view(-1)[pos] = torch.rand(10, generator=g) * 4.0
    logits[2] = torch.randn((C, H, W), generator=g) * 2.0  # image 2: the fast path
    size = torch.randn((B, H, W, 2), generator=g)
    offset = torch.rand((B, H, W, 2), generator=g)
    dec = DeviceDecoder(B, C, H, W, K, torch.device("cuda"))
    for order in ([0, 1, 2], [2, 0, 1], [1, 2, 0]):
        lg = logits[order]
        rec, cnt = dec(lg.cuda(), size.cuda(), offset.cuda(), None, 0, 4, 80, 120, 0.0)
        rec = rec.cpu().numpy()
        nms = oracle.heatmap_nms(torch.sigmoid(lg), 3).reshape(B, -1).numpy()
        ref_s, ref_i = _tie_rule_topk(nms, K)
        np.testing.assert_array_equal(rec[..., 7].astype(np.int64), ref_i)
        np.testing.assert_allclose(rec[..., 1], ref_s, rtol=0, atol=1e-6)
        assert (cnt.cpu().numpy() == K).all()


def test_decode_nhwc_aligned_heads_match_nchw():
    """The engine's head tensor layout (NHWC, 4 heat channels first, pixel stride a multiple of
    4 floats: the float4 fill path of peak_scan) decodes exactly as the plain NCHW tensors."""
    from tauv_vision_amd.decode import DeviceDecoder
    g = torch.Generator().manual_seed(11)
    B, C, H, W, K = 5, 4, 60, 80, 100
    logits = torch.randn((B, C, H, W), generator=g) * 2.0
    size = torch.randn((B, H, W, 2), generator=g)
    offset = torch.rand((B, H, W, 2), generator=g)
    nhwc = torch.cat([logits.permute(0, 2, 3, 1), size, offset], dim=3).contiguous().cuda()  # 8 channels
    dec = DeviceDecoder(B, C, H, W, K, torch.device("cuda"))
    r1, c1 = dec(nhwc[..., 0:4].permute(0, 3, 1, 2), nhwc[..., 4:6], nhwc[..., 6:8], None, 0, 4, 240, 320, 0.2)
    r1, c1 = r1.cpu().numpy().copy(), c1.cpu().numpy().copy()
    r2, c2 = dec(logits.cuda(), size.cuda(), offset.cuda(), None, 0, 4, 240, 320, 0.2)
    np.testing.assert_array_equal(r1, r2.cpu().numpy())
    np.testing.assert_array_equal(c1, c2.cpu().numpy())


@pytest.mark.parametrize("B,C,H,W,K,scale", [
    (2, 4, 120, 160, 300, 3.0),     # K > 256: candidates over several threads each
    (1, 4, 400, 400, 1024, 3.0),    # ~10^5 appended keys: the select streams them from global memory
    (2, 2, 40, 50, 1000, 0.05),     # < K positive peaks per image with K > 256: streaming fallback carry
    (3, 1, 7, 9, 20, 2.0),          # one tile per image: the scanning workgroup selects itself
])
def test_decode_single_launch_large_k_and_streaming(B, C, H, W, K, scale):
    """tv_decode's single launch (the image's last scan workgroup selects) against the CPU oracle at
    K beyond the direct-rank cap, an image whose kept keys exceed the register cache, images with
    fewer positive peaks than K, and a one-tile image; called twice through one workspace (the
    counters it leaves at zero)."""
    from tauv_vision_amd.decode import DeviceDecoder
    g = torch.Generator().manual_seed(B * 1000 + K)
    logits = torch.randn((B, C, H, W), generator=g) * scale
    if scale < 1.0:  # few positive peaks: a handful of raised cells on a saturated-to-zero map
        logits.fill_(-200.0)
        for b in range(B):
            pos = torch.randperm(C * H * W, generator=g)[:40]
            logits[b].view(-1)[pos] = torch.rand(40, generator=g) * 4.0
    size = torch.randn((B, H, W, 2), generator=g)
    offset = torch.rand((B, H, W, 2), generator=g)
    dec = DeviceDecoder(B, C, H, W, K, torch.device("cuda"))
    nms = oracle.heatmap_nms(torch.sigmoid(logits), 3).reshape(B, -1).numpy()
    ref_s, ref_i = _tie_rule_topk(nms, K)
    for _ in range(2):
        rec, cnt = dec(logits.cuda(), size.cuda(), offset.cuda(), None, 0, 4, 4 * H, 4 * W, 0.0)
        rec = rec.cpu().numpy()
        np.testing.assert_array_equal(rec[..., 7].astype(np.int64), ref_i)
        np.testing.assert_allclose(rec[..., 1], ref_s, rtol=0, atol=1e-6)
        assert (cnt.cpu().numpy() == K).all()
    assert int(dec.ws[:8 * B].view(torch.int32).abs().sum()) == 0, "counters not left at zero"


def test_decode_graph_replay():
    """DeviceDecoder captured in a HIP graph: replays on new heatmaps give the eager records (the
    single launch resets its own counters; no memset node)."""
    from tauv_vision_amd.decode import DeviceDecoder
    B, C, H, W, K = 4, 4, 120, 160, 100
    g = torch.Generator().manual_seed(3)
    heat = (torch.randn((B, C, H, W), generator=g) * 2.0).cuda()
    size = torch.randn((B, H, W, 2), generator=g).cuda()
    offset = torch.rand((B, H, W, 2), generator=g).cuda()
    dec = DeviceDecoder(B, C, H, W, K, torch.device("cuda"))
    dec(heat, size, offset, None, 0, 4, 480, 640, 0.3)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            rec_g, cnt_g = dec(heat, size, offset, None, 0, 4, 480, 640, 0.3)
    for seed in (10, 11, 12):
        heat.copy_(torch.randn((B, C, H, W), generator=torch.Generator().manual_seed(seed)).cuda() * 2.0)
        rec_g.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        got_r, got_c = rec_g.cpu().clone(), cnt_g.cpu().clone()
        ref = DeviceDecoder(B, C, H, W, K, torch.device("cuda"))
        r2, c2 = ref(heat, size, offset, None, 0, 4, 480, 640, 0.3)
        assert torch.equal(got_c, c2.cpu())
        assert torch.equal(got_r.nan_to_num(-7.0), r2.cpu().nan_to_num(-7.0))


def test_decode_workspace_shared_across_batch_sizes_and_geometries():
    """One zero-filled workspace, sized for the largest call, serves calls at other B and heatmap
    geometries in any order (the per-image counters sit at fixed offsets, so a smaller-B call's
    keys never land on a larger-B call's counters): B=8, B=2, another geometry, B=8 again."""
    from tauv_vision_amd.decode import DeviceDecoder
    dev = torch.device("cuda")
    calls = [(8, 4, 120, 160, 100), (2, 4, 120, 160, 100), (3, 2, 200, 96, 300), (8, 4, 120, 160, 100)]
    decs = [DeviceDecoder(*c, dev) for c in calls]
    shared = torch.zeros(max(d.ws_bytes for d in decs), dtype=torch.uint8, device=dev)
    for i, ((B, C, H, W, K), dec) in enumerate(zip(calls, decs)):
        dec.ws, dec.ws_bytes = shared, shared.numel()
        g = torch.Generator().manual_seed(900 + i)
        logits = torch.randn((B, C, H, W), generator=g) * 2.5
        size = torch.randn((B, H, W, 2), generator=g)
        offset = torch.rand((B, H, W, 2), generator=g)
        rec, cnt = dec(logits.cuda(), size.cuda(), offset.cuda(), None, 0, 4, 4 * H, 4 * W, 0.0)
        rec = rec.cpu().numpy()
        ref_s, ref_i = _tie_rule_topk(oracle.heatmap_nms(torch.sigmoid(logits), 3).reshape(B, -1).numpy(), K)
        np.testing.assert_array_equal(rec[..., 7].astype(np.int64), ref_i)
        np.testing.assert_allclose(rec[..., 1], ref_s, rtol=0, atol=1e-6)
        assert (cnt.cpu().numpy() == K).all()
    assert int(shared[:8 * 8].view(torch.int32).abs().sum()) == 0, "counters not left at zero"
