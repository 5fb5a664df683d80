"""convt3.hip: the YOLACT protonet's ConvTranspose2d(F, F, 3, stride 2, padding 1, output_padding 1)
+ LeakyReLU (masknet.py:21,33, `_upsample_layer_{1,2}`) with its four output phases in one launch
over a shared input halo (the round-4 engine ran them as four phase GEMMs on conv_pipe).

Checked:
  * single layers through tv_diag_convt3 against torch.nn.functional.conv_transpose2d (the
    reference's own op) on dtype-rounded operands: both protonet sizes (69x69, 138x138 inputs of
    the 550x550 config), frames smaller than a tile, ragged tile edges, forced tile shapes whose
    fragments span several input rows, every activation, channel counts 32..256 / 64..192;
  * the engine takes it for both up-sampling layers (the other three phase ops launch nothing);
  * the protonet forward against the same forward with the kernel off (knob TV_CT3=0: the phase
    GEMMs) within the low-precision tolerance, and repeated forwards bit-identical. The reference
    goldens run through the default path in test_yolact.py.
"""
import ctypes

import pytest
import torch

from recipe import protonet_case, protonet_inputs

pytestmark = pytest.mark.gpu

SCALES = (24, 48, 96, 192, 384)
VAR = (0.1, 0.2)


def _diag(x, w, b, act, precision, tile=(0, 0), pad=8):
    """x [B, C, H, W] fp32 (already rounded), w [C, N, 3, 3], b [N] -> [B, N, 2H, 2W] fp32."""
    from tauv_vision_amd import _lib
    dt, code = {"fp16": (torch.float16, 1), "bf16": (torch.bfloat16, 2)}[precision]
    B, C, H, W = x.shape
    N = w.shape[1]
    dev = x.permute(0, 2, 3, 1).to(dt).cuda().contiguous()
    out = torch.full((B, 2 * H, 2 * W, N + pad), float("nan"), dtype=dt, device="cuda")
    wc, bc = w.float().contiguous(), b.float().contiguous()
    L = _lib.lib()
    _lib.check(L.tv_diag_convt3(ctypes.c_void_p(dev.data_ptr()), B, H, W, C, C, ctypes.c_void_p(wc.data_ptr()),
                                ctypes.c_void_p(bc.data_ptr()), N, act, code, tile[0], tile[1],
                                ctypes.c_void_p(out.data_ptr()), N + pad, _lib.stream_of(out.device)), "convt3")
    assert torch.isnan(out[..., N:].float()).all(), "wrote past the N output channels"
    return out[..., :N].float().cpu().permute(0, 3, 1, 2)


def _ref(x, w, b, act):
    y = torch.nn.functional.conv_transpose2d(x, w, b, stride=2, padding=1, output_padding=1)
    return torch.relu(y) if act == 1 else torch.nn.functional.leaky_relu(y, 0.01) if act == 2 else y


# (B, C, H, W, N, act, (tile_w, tile_h)): the protonet's two layers (F = 256, the 550x550 config),
# its 9x17 test case (F = 64), frames smaller than one tile, forced tile shapes (exact 16x16,
# fragments over several rows at 7 columns, the widest tile), wide N
SHAPES = [
    (1, 256, 69, 69, 256, 2, (0, 0)),
    (1, 256, 138, 138, 256, 2, (0, 0)),
    (2, 64, 9, 17, 64, 2, (0, 0)),
    (3, 32, 5, 37, 128, 0, (0, 0)),
    (1, 96, 16, 16, 64, 1, (16, 16)),
    (2, 64, 23, 11, 192, 2, (23, 11)),
    (1, 64, 40, 9, 64, 2, (7, 32)),
    (1, 128, 3, 200, 64, 2, (60, 4)),
    (2, 64, 1, 1, 64, 2, (0, 0)),
]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("B,C,H,W,N,act,tile", SHAPES)
def test_convt3_single_layer_vs_torch(B, C, H, W, N, act, tile, precision):
    g = torch.Generator().manual_seed(H * 1000 + W + N + C)
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[precision]
    x = torch.randn(B, C, H, W, generator=g).to(dt).float()
    w = (torch.randn(C, N, 3, 3, generator=g) / (2.25 * C) ** 0.5).to(dt).float()
    b = torch.randn(N, generator=g) * 0.1
    got = _diag(x, w, b, act, precision, tile)
    ref = _ref(x, w, b, act)
    eps = {"fp16": 2.0 ** -10, "bf16": 2.0 ** -7}[precision]
    err = (got - ref).abs()
    assert bool((err <= eps * ref.abs() + 2e-3).all()), f"max err {float(err.max()):.3e}"


def test_convt3_rejects_unsupported():
    from tauv_vision_amd import _lib
    x = torch.zeros(1, 48, 4, 4)
    w = torch.zeros(48, 64, 3, 3)
    with pytest.raises(ValueError):
        _diag(x, w, torch.zeros(64), 0, "fp16")  # 48 channels: not a multiple of 32
    with pytest.raises(ValueError):
        _diag(torch.zeros(1, 64, 4, 4), torch.zeros(64, 64, 3, 3), torch.zeros(64), 0, "fp16", (64, 8))  # tile
    assert _lib.lib() is not None


def _masknet(F, k, precision, state):
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    m = Masknet(YolactConfig(640, 360, SCALES, (1,), VAR, feature_depth=F, n_prototype_masks=k), precision=precision)
    m.load_state_dict(state)
    return m


def _knobs(monkeypatch, knobs):
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", dict(knobs))


def test_convt3_selection(monkeypatch):
    _knobs(monkeypatch, {})
    c = protonet_case("protonet_f256_k8_b1_69x69")
    sd, x = protonet_inputs(c)
    m = _masknet(256, 8, "fp16", sd)
    eng = m.engine(torch.device("cuda", 0), 69, 69)
    xs = x.cuda().float().contiguous()
    kern = {label: k for label, _, _, k in eng.profile(xs, eng.alloc_out(1))}
    for up in ("_upsample_layer_1", "_upsample_layer_2"):
        assert kern[f"{up} phase (0,0) + LeakyReLU"].startswith("tv::ct3::convt3<"), kern
        for ph in ("(0,1)", "(1,0)", "(1,1)"):
            assert kern[f"{up} phase {ph} + LeakyReLU"].startswith("(fused"), kern
    assert not any(k.startswith("tv::pipe::conv_pipe<") and k.endswith(", 1>") for k in kern.values()), kern


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_convt3_forward_matches_phase_gemms_and_is_deterministic(monkeypatch, precision):
    tol = {"fp16": 8e-4, "bf16": 6e-3}[precision]
    c = protonet_case("protonet_f64_k16_b1_9x17")
    sd, _ = protonet_inputs(c)
    x = torch.randn(5, 64, 9, 17, generator=torch.Generator().manual_seed(11)).cuda()
    _knobs(monkeypatch, {})
    m = _masknet(64, 16, precision, sd)
    runs = [m(x) for _ in range(3)]
    for r in runs[1:]:
        assert torch.equal(r, runs[0])
    _knobs(monkeypatch, {"TV_CT3": "0"})
    ref = _masknet(64, 16, precision, sd)(x)
    scale = max(1.0, float(ref.abs().max()))
    assert float((runs[0] - ref).abs().max()) <= tol * scale
