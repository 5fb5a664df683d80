"""conv_small.hip: the narrow-channel 3x3 convs of DLA-34's full-resolution base levels
(centerpoint_dla.py:242-246 `_make_conv_level`: level0 16 -> 16 at 480x640, level1 16 -> 32
stride 2, level2's first conv 32 -> 64 stride 2), in both variants: per-lane register gathers
(variant 0) and LDS-halo tiles, one per workgroup (variant 1) or on a persistent grid (variant 2);
the engine runs the persistent halo tiles (knob TV_CSM_HALO forces another variant).

Checked:
  * single layers through tv_diag_conv_small against torch.nn.functional.conv2d on dtype-rounded
    operands: every supported (C, N, stride), frames smaller than a halo tile, ragged tile edges,
    channel-sliced input (ldc > C) and output (out_ldc > N: nothing written past N), every
    activation; the two variants bit-identical (the same MFMA sequence over the same K order);
  * DLA-34 forwards with each variant forced bit-identical, and the engine's kernel names showing
    which variant ran; by default (knob unset) all three layers run the halo tiles.
"""
import ctypes

import pytest
import torch

from recipe import seeded_u8_frames, normalize

pytestmark = pytest.mark.gpu


def _diag(x, w, b, stride, act, precision, variant, ldc_pad=0, pad=8):
    """x [B, C, H, W] fp32 (already rounded), w [N, C, 3, 3], b [N] -> [B, N, Ho, Wo] fp32."""
    from tauv_vision_amd import _lib
    dt, code = {"fp16": (torch.float16, 1), "bf16": (torch.bfloat16, 2)}[precision]
    B, C, H, W = x.shape
    N = w.shape[0]
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    xs = torch.full((B, H, W, C + ldc_pad), float("nan"), dtype=dt)
    xs[..., :C] = x.permute(0, 2, 3, 1).to(dt)
    dev = xs.cuda().contiguous()
    out = torch.full((B, Ho, Wo, N + pad), float("nan"), dtype=dt, device="cuda")
    wc, bc = w.float().contiguous(), b.float().contiguous()
    L = _lib.lib()
    _lib.check(L.tv_diag_conv_small(ctypes.c_void_p(dev.data_ptr()), B, H, W, C, C + ldc_pad,
                                    ctypes.c_void_p(wc.data_ptr()), ctypes.c_void_p(bc.data_ptr()), N, stride, act,
                                    code, variant, ctypes.c_void_p(out.data_ptr()), N + pad,
                                    _lib.stream_of(out.device)), "conv_small")
    assert torch.isnan(out[..., N:].float()).all(), "wrote past the N output channels"
    return out[..., :N].float().cpu().permute(0, 3, 1, 2)


def _ref(x, w, b, stride, act):
    y = torch.nn.functional.conv2d(x, w, b, stride=stride, padding=1)
    return torch.relu(y) if act == 1 else torch.nn.functional.leaky_relu(y, 0.01) if act == 2 else y


# (B, C, N, stride, H, W, act, ldc_pad): DLA-34's three layers at a reduced frame, frames smaller
# than one halo tile, ragged edges in both directions, odd sizes at stride 2, sliced channels
SHAPES = [
    (2, 16, 16, 1, 48, 64, 1, 0),
    (1, 16, 32, 2, 48, 64, 1, 0),
    (1, 32, 64, 2, 24, 32, 1, 0),
    (1, 32, 32, 1, 17, 70, 2, 0),
    (3, 16, 16, 1, 5, 9, 0, 0),
    (1, 16, 32, 1, 13, 67, 1, 8),
    (2, 16, 16, 2, 19, 33, 2, 0),
    (1, 16, 32, 2, 35, 81, 1, 16),
    (2, 32, 64, 2, 9, 131, 0, 8),
    (1, 16, 16, 1, 1, 1, 1, 0),
]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("B,C,N,stride,H,W,act,ldc_pad", SHAPES)
def test_conv_small_vs_torch_both_variants(B, C, N, stride, H, W, act, ldc_pad, precision):
    g = torch.Generator().manual_seed(H * 1000 + W + N + C + stride)
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[precision]
    x = torch.randn(B, C, H, W, generator=g).to(dt).float()
    w = (torch.randn(N, C, 3, 3, generator=g) / (9.0 * C) ** 0.5).to(dt).float()
    b = torch.randn(N, generator=g) * 0.1
    ref = _ref(x, w, b, stride, act)
    eps = {"fp16": 2.0 ** -10, "bf16": 2.0 ** -7}[precision]
    got = [_diag(x, w, b, stride, act, precision, v, ldc_pad) for v in (0, 1, 2)]
    for v, o in enumerate(got):
        err = (o - ref).abs()
        assert bool((err <= eps * ref.abs() + 2e-3).all()), f"variant {v}: max err {float(err.max()):.3e}"
    assert torch.equal(got[0], got[1]), "register-gather and LDS-halo variants differ"
    assert torch.equal(got[0], got[2]), "register-gather and persistent LDS-halo variants differ"


def test_conv_small_rejects_unsupported():
    x = torch.zeros(1, 24, 8, 8)
    with pytest.raises(ValueError):
        _diag(x, torch.zeros(16, 24, 3, 3), torch.zeros(16), 1, 0, "fp16", 1)  # 24 input channels
    with pytest.raises(ValueError):
        _diag(torch.zeros(1, 32, 8, 8), torch.zeros(64, 32, 3, 3), torch.zeros(64), 1, 0, "fp16", 1)  # 32->64 s1


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_dla34_forward_halo_variant_bit_identical(monkeypatch, precision):
    import test_gpu_dla34 as dla
    import test_gpu_forward as fwd
    from tauv_vision_amd import engine as E
    x = normalize(seeded_u8_frames(3, 480, 640, seed=23).permute(0, 3, 1, 2).float() / 255.0).cuda()
    res = {}
    for halo in ("0", "1", "2"):
        monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_CSM_HALO": halo})
        model = dla.build("b1_480x640_kp", precision)[0]
        pred = model(x)
        eng = model.engine(torch.device("cuda", 0), 480, 640)
        kern = [k for _, _, _, k in eng.profile(x, eng.alloc_out(3))]
        want = "tv::csm::conv_small_halo<" if halo != "0" else "tv::csm::conv_small<"
        assert sum(k.startswith(want) for k in kern) >= 3, kern
        res[halo] = {f: getattr(pred, f).detach().float().cpu() for f in fwd.FIELDS if getattr(pred, f) is not None}
    for f in res["0"]:
        assert torch.equal(res["0"][f], res["1"][f]), f
        assert torch.equal(res["0"][f], res["2"][f]), f


def test_default_variant_choice(monkeypatch):
    import test_gpu_dla34 as dla
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", {})
    x = normalize(seeded_u8_frames(2, 480, 640, seed=24).permute(0, 3, 1, 2).float() / 255.0).cuda()
    model = dla.build("b1_480x640_kp", "fp16")[0]
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    kern = [k for _, _, _, k in eng.profile(x, eng.alloc_out(2))]
    halo = [k for k in kern if k.startswith("tv::csm::conv_small_halo<")]
    assert len(halo) >= 3 and not any(k.startswith("tv::csm::conv_small<") for k in kern), kern
