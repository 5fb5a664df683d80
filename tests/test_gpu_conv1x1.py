"""conv1x1.hip: the streaming stride-1 1x1 conv over concatenated inputs (the DLA Roots,
dla.py:58-76) that the engine picks where conv_pipe used to run (the large levels of a batch:
at B=1 those layers are on conv_lat's latency path) — the kernel the engine selects, and its
results against the pipelined GEMM (diagnostic knob TV_C1X1=0): the same fp32 products summed in
another order, so within the low-precision tolerance of test_gpu_forward.py."""
import pytest
import torch

from recipe import seeded_u8_frames, normalize

import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu


def _knobs(monkeypatch, knobs):
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", dict(knobs))


def _run(monkeypatch, knobs, builder, x):
    _knobs(monkeypatch, knobs)
    model = builder()
    pred = model(x)
    eng = model.engine(torch.device("cuda", 0), x.shape[-2], x.shape[-1])
    kern = {lab: k for lab, _, _, k in eng.profile(x, eng.alloc_out(x.shape[0]))}
    return {f: getattr(pred, f).detach().float().cpu() for f in fwd.FIELDS if getattr(pred, f) is not None}, kern


@pytest.mark.parametrize("name", ["r18_c128_b1_480x640", "dla34:b1_480x640_kp"])
@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_conv1x1_stream_matches_pipe(monkeypatch, name, precision):
    if name.startswith("dla34:"):
        import test_gpu_dla34 as dla
        name = name.split(":", 1)[1]
        builder = lambda: dla.build(name, precision)[0]  # noqa: E731
        tol = dla.TOL[precision]
    else:
        builder = lambda: fwd.build(name, precision)[0]  # noqa: E731
        tol = fwd.TOL[precision]
    x = normalize(seeded_u8_frames(16, 480, 640, seed=16).permute(0, 3, 1, 2).float() / 255.0).cuda()
    ref, kref = _run(monkeypatch, {"TV_C1X1": "0"}, builder, x)
    assert not any("c1x1" in k for k in kref.values())
    got, kern = _run(monkeypatch, {}, builder, x)
    assert any(k.startswith("tv::c1x1::conv1x1_stream<") for k in kern.values()), kern
    for f in ref:
        scale = max(1.0, float(ref[f].abs().max()))
        err = float((got[f] - ref[f]).abs().max())
        assert err <= tol * scale, f"{name} {precision} {f}: {err:.3e}"


def test_wide_roots_on_conv1x1_stream(monkeypatch):
    """DLA-34's level-4 Roots (256 output channels) run as 128-channel slices of conv1x1_stream;
    knob TV_C1X1=2 keeps layers wider than 128 channels on conv_pipe, with the same outputs within
    the low-precision tolerance."""
    import test_gpu_dla34 as dla
    builder = lambda: dla.build("b1_480x640_kp", "fp16")[0]  # noqa: E731
    x = normalize(seeded_u8_frames(16, 480, 640, seed=17).permute(0, 3, 1, 2).float() / 255.0).cuda()
    ref, kref = _run(monkeypatch, {"TV_C1X1": "2"}, builder, x)
    got, kern = _run(monkeypatch, {}, builder, x)
    wide = [lab for lab, k in kern.items() if "level4" in lab and k.startswith("tv::c1x1::")]
    assert wide, kern
    assert not any(kref[lab].startswith("tv::c1x1::") for lab in wide), kref
    for f in ref:
        scale = max(1.0, float(ref[f].abs().max()))
        assert float((got[f] - ref[f]).abs().max()) <= dla.TOL["fp16"] * scale, f


def _diag_conv1x1(xs, w, b, act, precision, out_ldc=None):
    """xs: list of [M, C_k] fp32 (already rounded) segments; w [N, sum C] fp32; -> [M, N] fp32 via
    tv_diag_conv1x1 (conv1x1_stream with the engine's Root packing)."""
    import ctypes
    from tauv_vision_amd import _lib
    dt, code = {"fp16": (torch.float16, 1), "bf16": (torch.bfloat16, 2)}[precision]
    M, N = xs[0].shape[0], w.shape[0]
    # every segment in its own wider row (ldc > C) to cover the strided-source path
    dev = [torch.zeros(M, x.shape[1] + 8 * (k + 1), dtype=dt, device="cuda") for k, x in enumerate(xs)]
    for d, x in zip(dev, xs):
        d[:, :x.shape[1]] = x.to(dt).cuda()
    ldo = out_ldc or N
    out = torch.full((M, ldo), float("nan"), dtype=dt, device="cuda")
    ptrs = (ctypes.c_void_p * len(xs))(*[d.data_ptr() for d in dev])
    Cs = (ctypes.c_int32 * len(xs))(*[x.shape[1] for x in xs])
    lds = (ctypes.c_int32 * len(xs))(*[d.shape[1] for d in dev])
    wc, bc = w.float().contiguous(), b.float().contiguous()
    L = _lib.lib()
    _lib.check(L.tv_diag_conv1x1(ptrs, Cs, lds, len(xs), M, ctypes.c_void_p(wc.data_ptr()),
                                 ctypes.c_void_p(bc.data_ptr()), N, act, code, ctypes.c_void_p(out.data_ptr()), ldo,
                                 _lib.stream_of(out.device)), "conv1x1")
    return out[:, :N].float().cpu(), out[:, N:].float().cpu()


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("M,Cs,N,act", [
    (8 * 37 + 5, [128, 128], 8, 1),         # one 32-pixel tile's tail; N = 8 (a quarter fragment)
    (1021, [64, 192, 128], 96, 2),          # odd M, three segments of different width, leaky
    (4099, [256], 192, 0),                  # two 128-channel slices, the second partial (64 of 128)
    (777, [128, 64], 320, 1),               # three slices, the last 64 wide; K = 192
    (33, [128, 128, 128], 512, 2),          # the widest layer it takes (DLA-34 level-4 Roots)
])
def test_conv1x1_stream_synthetic_shapes(M, Cs, N, act, precision):
    """conv1x1_stream against a torch fp32 cat + 1x1 conv + bias + activation on the shapes the
    engine's selector accepts but the model tests never run: M % 32 != 0 (the pixel tail), N > 128
    not a multiple of 128 (a partial last slice), 2-3 segments of different C / kbase, act 0/1/2."""
    g = torch.Generator().manual_seed(M + N)
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[precision]
    xs = [torch.randn(M, c, generator=g).to(dt).float() for c in Cs]
    K = sum(Cs)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt).float()
    b = torch.randn(N, generator=g) * 0.1
    ref = torch.cat(xs, 1) @ w.t() + b
    if act == 1:
        ref = torch.relu(ref)
    elif act == 2:
        ref = torch.nn.functional.leaky_relu(ref, 0.01)
    got, pad = _diag_conv1x1(xs, w, b, act, precision, out_ldc=N + 8)
    assert torch.isnan(pad).all(), "wrote past the N output channels"
    eps = {"fp16": 2.0 ** -10, "bf16": 2.0 ** -7}[precision]  # one output rounding
    err = (got - ref).abs()
    assert bool((err <= eps * ref.abs() + 1e-3).all()), f"max err {float(err.max()):.3e}"
