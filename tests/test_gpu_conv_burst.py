"""conv_burst.hip (the one-shot small-level conv: a workgroup's whole operand set requested at once,
weights in registers, the input window staged in LDS, K split over four waves and summed in wave
order) — the deep DLA levels of dla.py:79-135 (Trees, their Roots dla.py:58-76 and ResidualBlocks
with the fused 1x1 conv_residual dla.py:8-52) and the IDAUp projections / outputs (dla.py:212-284).

Checked:
  * which layers it takes: at B=32 the stride-1 deep levels; the strided 3x3 stay on conv_lat;
  * against the reference goldens at B = 1 and 3 with every representable layer forced onto it
    (diagnostic knob TV_LAT_UNITS huge: the 60x80 levels too, whose 3-row windows are the largest),
    the golden frame at the last batch position (a partial last pixel tile);
  * against conv_lat (knob TV_BURST=0): the same fp32 products summed in another order, within the
    low-precision tolerance; repeated forwards bit-identical;
  * DLA-34 (its 128-channel levels on the burst kernel, the 256 / 512-channel ones on conv_lat)
    against its goldens.
"""
import pytest
import torch

from helpers import golden, case_input, dla34_input

import test_gpu_dla34 as dla
import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu

NAME = "r18_c128_b1_480x640"


def _knobs(monkeypatch, knobs):
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", dict(knobs))


def _kernels(model, B):
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    frames = torch.zeros((B, 480, 640, 3), dtype=torch.uint8, device="cuda")
    return {label: k for label, _, _, k in eng.profile(frames, eng.alloc_out(B))}


def test_burst_selection(monkeypatch):
    """By default the one-shot kernel takes the layers whose tiles are all resident at once with a
    window of <= 64 KiB: at B=32 the 8x10 and 4x5 levels and the 15x20 layers that fit one round, at B=1
    everything below 60x80 (its 80-column windows keep conv_lat); strided 3x3 stay on conv_lat."""
    _knobs(monkeypatch, {})
    model, _, _, _ = fwd.build(NAME, "fp16")
    kern = _kernels(model, 32)
    for lab in ("backbone.dla_down.tree_layers.3.tree_l.tree_l.conv2+conv_residual",
                "backbone.dla_down.tree_layers.4.tree_r.root.conv",
                "backbone.multi_ida_up.ida_up_layers.0.projection_layers.4.0"):
        assert kern[lab].startswith("tv::burst::conv_burst<"), (lab, kern[lab])
    assert kern["backbone.dla_down.tree_layers.3.tree_l.tree_l.conv1"].startswith("tv::lat::conv_lat<"), kern
    # 15x20 conv2 + residual: a 58 KiB staging, two workgroups per CU, 640 tiles -> two rounds
    assert kern["backbone.dla_down.tree_layers.2.tree_l.tree_r.conv2+conv_residual"].startswith("tv::lat::conv_lat<"), kern
    k1 = _kernels(model, 1)
    assert k1["backbone.dla_down.tree_layers.1.tree_l.tree_r.conv1"].startswith("tv::burst::conv_burst<"), k1
    assert k1["backbone.dla_down.tree_layers.0.tree_l.tree_r.conv1"].startswith("tv::lat::conv_lat<"), k1


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("B", [1, 3])
def test_burst_everywhere_matches_reference(monkeypatch, precision, B):
    _knobs(monkeypatch, {"TV_LAT_UNITS": str(10 ** 9), "TV_BURST": "2"})
    model, _, _, _ = fwd.build(NAME, precision)
    kern = _kernels(model, B)
    burst = [lab for lab, k in kern.items() if k.startswith("tv::burst::conv_burst<")]
    assert len(burst) >= 50, kern
    assert any(".tree_layers.0." in lab for lab in burst), burst  # the 60x80 level (3-row windows)
    img = case_input(NAME).cuda()
    pred = model(torch.cat([torch.flip(img, [-1])] * (B - 1) + [img], 0))
    g = golden(f"model_{NAME}")
    for f in ("heatmap", "size", "offset"):
        ref = g[f]
        got = getattr(pred, f)[B - 1:].detach().float().cpu().numpy()
        scale = max(1.0, float(abs(ref).max()))
        assert float(abs(got - ref).max()) <= fwd.TOL[precision] * scale, f


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_burst_matches_conv_lat_and_is_deterministic(monkeypatch, precision):
    img = case_input(NAME).cuda()
    x = torch.cat([img, torch.flip(img, [-2]), torch.flip(img, [-1])], 0)
    _knobs(monkeypatch, {})
    model, _, _, _ = fwd.build(NAME, precision)
    runs = [model(x) for _ in range(3)]
    for f in ("heatmap", "size", "offset"):
        for r in runs[1:]:
            assert torch.equal(getattr(r, f), getattr(runs[0], f)), f
    _knobs(monkeypatch, {"TV_BURST": "0"})
    ref_model, _, _, _ = fwd.build(NAME, precision)
    ref = ref_model(x)
    for f in ("heatmap", "size", "offset"):
        a, b = getattr(runs[0], f).float(), getattr(ref, f).float()
        scale = max(1.0, float(b.abs().max()))
        assert float((a - b).abs().max()) <= fwd.TOL[precision] * scale, f


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_burst_dla34_matches_reference(monkeypatch, precision):
    _knobs(monkeypatch, {})
    name = "b1_480x640_kp"
    model, _, _, _ = dla.build(name, precision)
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    x = dla34_input(name).cuda()
    kern = {label: k for label, _, _, k in eng.profile(x, eng.alloc_out(1))}
    assert any(k.startswith("tv::burst::conv_burst<") for k in kern.values()), kern
    dla._cmp(model(x), golden(f"dla34_{name}"), dla.TOL[precision])


def _diag_burst(segs, B, Ho, Wo, w, b, act, precision):
    """segs: list of (x [B, C, H, W] fp32 rounded, kernel, stride); w [N, K] fp32 (K segment-major,
    tap-major, channel-minor); -> [B, N, Ho, Wo] fp32 via tv_diag_conv_burst."""
    import ctypes
    from tauv_vision_amd import _lib
    dt, code = {"fp16": (torch.float16, 1), "bf16": (torch.bfloat16, 2)}[precision]
    dev = []
    geom = []
    for x, k, st in segs:
        _, C, H, W = x.shape
        dev.append(x.permute(0, 2, 3, 1).to(dt).cuda().contiguous())
        geom += [H, W, C, C, k, st]
    N = w.shape[0]
    out = torch.full((B, Ho, Wo, N + 8), float("nan"), dtype=dt, device="cuda")
    ptrs = (ctypes.c_void_p * len(segs))(*[d.data_ptr() for d in dev])
    g = (ctypes.c_int32 * len(geom))(*geom)
    wc, bc = w.float().contiguous(), b.float().contiguous()
    L = _lib.lib()
    _lib.check(L.tv_diag_conv_burst(ptrs, g, len(segs), B, Ho, Wo, ctypes.c_void_p(wc.data_ptr()),
                                    ctypes.c_void_p(bc.data_ptr()), N, act, code, ctypes.c_void_p(out.data_ptr()), N + 8,
                                    _lib.stream_of(out.device)), "conv_burst")
    assert torch.isnan(out[..., N:].float()).all(), "wrote past the N output channels"
    return out[..., :N].float().cpu().permute(0, 3, 1, 2)


def _ref(segs, w, b, act):
    y, k0 = None, 0
    N = w.shape[0]
    for x, k, st in segs:
        C = x.shape[1]
        wk = w[:, k0:k0 + k * k * C].reshape(N, k, k, C).permute(0, 3, 1, 2)
        k0 += k * k * C
        t = torch.nn.functional.conv2d(x, wk, stride=st, padding=k // 2)
        y = t if y is None else y + t
    y = y + b.view(1, -1, 1, 1)
    return torch.relu(y) if act == 1 else torch.nn.functional.leaky_relu(y, 0.01) if act == 2 else y


# (B, Ho, Wo, [(C, kernel, stride)], N, act): the Tree conv2 + fused stride-2 1x1 residual, plain
# 3x3 at every deep level incl. 60x80 (the largest window) and a 4x5 frame (tile > frame), Roots of
# 2 and 3 children, a 256-channel 1x1 (two LDS planes), partial channel tiles
SHAPES = [
    (2, 15, 20, [(128, 3, 1)], 128, 1),
    (2, 15, 20, [(128, 3, 1), (128, 1, 2)], 128, 1),
    (3, 4, 5, [(128, 3, 1)], 128, 2),
    (1, 60, 80, [(128, 3, 1)], 96, 0),
    (2, 8, 10, [(128, 1, 1), (128, 1, 1), (128, 1, 1)], 128, 1),
    (1, 30, 40, [(256, 1, 1), (128, 1, 1)], 64, 1),
    (2, 8, 10, [(128, 3, 1), (128, 1, 1)], 40, 1),
]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("B,Ho,Wo,segspec,N,act", SHAPES)
def test_burst_single_layer_vs_torch(B, Ho, Wo, segspec, N, act, precision):
    g = torch.Generator().manual_seed(Ho * 100 + Wo + N)
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[precision]
    segs = []
    for C, k, st in segspec:
        H, W = (Ho - 1) * st + 1 + (st - 1), (Wo - 1) * st + 1 + (st - 1)
        segs.append((torch.randn(B, C, H, W, generator=g).to(dt).float(), k, st))
    K = sum(k * k * C for C, k, _ in segspec)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt).float()
    b = torch.randn(N, generator=g) * 0.1
    got = _diag_burst(segs, B, Ho, Wo, w, b, act, precision)
    ref = _ref(segs, w, b, act)
    eps = {"fp16": 2.0 ** -10, "bf16": 2.0 ** -7}[precision]
    err = (got - ref).abs()
    assert bool((err <= eps * ref.abs() + 2e-3).all()), f"max err {float(err.max()):.3e}"
