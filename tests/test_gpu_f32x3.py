"""conv_pipe X3 (knob TV_F32X3 on fp32 engines): the fp32 convolutions' products as three fp16 MFMAs
(a_hi*b_hi + a_hi*b_lo + a_lo*b_hi, hi = fp16(x), lo = fp16(x - hi): ~22-bit operands, fp32
accumulation) against the reference goldens at the fp32 path's own tolerances (test_gpu_forward.py
/ test_gpu_dla34.py: 1e-4 of the output scale), and against the exact-fp32 engine."""
import pytest
import torch

from helpers import golden, case_input, dla34_input

import test_gpu_dla34 as dla
import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu

NAME = "r18_c128_b1_480x640"


def _kernels(model, B):
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    frames = torch.zeros((B, 480, 640, 3), dtype=torch.uint8, device="cuda")
    return {label: k for label, _, _, k in eng.profile(frames, eng.alloc_out(B))}


@pytest.mark.parametrize("precision,knobs", [("fp32x3", {}), ("fp32", {"TV_F32X3": "1", "TV_LAT_F32": "0"}),
                                             ("fp32", {"TV_F32X3": "1", "TV_PIPE_SPLIT": "0"})])
@pytest.mark.parametrize("B", [1, 3])
def test_f32x3_r18_golden(monkeypatch, precision, knobs, B):
    """precision="fp32x3" (the product path: tv_dtype TV_F32X3), and the diagnostic knob on an fp32
    engine with the deep levels on conv_pipe too / without split-K"""
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", knobs)
    model, _, _, _ = fwd.build(NAME, precision)
    kern = _kernels(model, B)
    assert sum(k.endswith(", true>") or ", true> split-K" in k for k in kern.values()) >= 3, kern
    img = case_input(NAME).cuda()
    pred = model(torch.cat([torch.flip(img, [-1])] * (B - 1) + [img], 0))
    g = golden(f"model_{NAME}")
    for f in ("heatmap", "size", "offset"):
        ref = g[f]
        got = getattr(pred, f)[B - 1:].detach().cpu().numpy()
        scale = max(1.0, float(abs(ref).max()))
        assert float(abs(got - ref).max()) <= fwd.TOL["fp32"] * scale, f
    monkeypatch.setattr(E, "_DIAG_KNOBS", {})
    exact = fwd.build(NAME, "fp32")[0](img)
    for f in ("heatmap", "size", "offset"):
        d = float((getattr(pred, f)[B - 1:] - getattr(exact, f)).abs().max())
        scale = max(1.0, float(getattr(exact, f).abs().max()))
        assert d <= 2e-5 * scale, (f, d)


def test_f32x3_dla34_golden():
    name = "b1_480x640_kp"
    model, _, _, _ = dla.build(name, "fp32x3")
    pred = model(dla34_input(name).cuda())
    dla._cmp(pred, golden(f"dla34_{name}"), dla.TOL["fp32"])
