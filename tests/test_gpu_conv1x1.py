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
