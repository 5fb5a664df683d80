"""conv_pipe.hip split-K (ksplit workgroups per 256 x 128 tile, the last to arrive sums the fp32
partial tiles in slice order, then bias + activation) against the reference goldens.

The engine picks it for the pipelined layers whose tiles fill the CUs badly — by default only on
the fp32 path (knob TV_PIPE_SPLIT=1), where a 15x20 level at B=1 is otherwise 2 tiles of 36
k-steps on 2 of 256 CUs (by default those deep levels take conv_lat.hip's 64-pixel tiles, split
as well: the last test; TV_LAT_F32=0 keeps them on conv_pipe). Checked: the fp32 engine splits the
deep layers, repeated
forwards are bit-identical (slice order fixed whichever workgroup arrives last), both the split
and the unsplit engine (TV_PIPE_SPLIT=0) match the golden within the fp32 tolerance of
test_gpu_forward.py / test_gpu_dla34.py, and the fp16 kernel instances (fp16 and fp32 outputs)
under TV_PIPE_SPLIT=2 with the halo / latency kernels off match at the fp16 tolerance.
"""
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


def _cmp_golden(pred, precision, B=1):
    g = golden(f"model_{NAME}")
    for f in ("heatmap", "size", "offset"):
        scale = max(1.0, float(abs(g[f]).max()))
        got = getattr(pred, f)[B - 1:].detach().cpu().numpy()
        assert float(abs(got - g[f]).max()) <= fwd.TOL[precision] * scale, f


def test_pipe_split_fp32_r18_b1(monkeypatch):
    from tauv_vision_amd import engine as E
    img = case_input(NAME).cuda()
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_LAT_F32": "0"})  # the deep levels on conv_pipe, split
    model, _, _, _ = fwd.build(NAME, "fp32")
    kern = _kernels(model, 1)
    split = [k for k in kern.values() if k.startswith("tv::pipe::conv_pipe<float, float, 0> split-K")]
    assert len(split) >= 20, kern
    runs = [model(img) for _ in range(3)]
    for f in ("heatmap", "size", "offset"):
        for r in runs[1:]:
            assert torch.equal(getattr(r, f), getattr(runs[0], f)), f
    _cmp_golden(runs[0], "fp32")
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_PIPE_SPLIT": "0", "TV_LAT_F32": "0"})
    model0, _, _, _ = fwd.build(NAME, "fp32")
    assert not any("split-K" in k for k in _kernels(model0, 1).values())
    ref = model0(img)
    g = golden(f"model_{NAME}")
    for f in ("heatmap", "size", "offset"):
        scale = max(1.0, float(abs(g[f]).max()))
        d = float((getattr(runs[0], f) - getattr(ref, f)).abs().max())
        assert d <= fwd.TOL["fp32"] * scale, (f, d)


@pytest.mark.parametrize("B", [2, 3])
def test_pipe_split_fp32_r18_batches(B):
    """Partial last tiles (M not a multiple of 256) and several frames per tile."""
    model, _, _, _ = fwd.build(NAME, "fp32")
    img = case_input(NAME).cuda()
    pred = model(torch.cat([torch.flip(img, [-1])] * (B - 1) + [img], 0))
    _cmp_golden(pred, "fp32", B)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_pipe_split_half_kernels(monkeypatch, precision):
    """Every layer the pipelined kernel represents on it (halo / latency / streaming kernels off),
    split wherever under-filled: the half-precision instances and the fp32-output heads."""
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_PIPE_SPLIT": "2", "TV_CONV3": "0", "TV_CONV3S2": "0", "TV_LAT": "0",
                                           "TV_C1X1": "0", "TV_HEADFUSE": "0", "TV_CONVT": "0", "TV_CT3": "0"})
    model, _, _, _ = fwd.build(NAME, precision)
    kern = _kernels(model, 1)
    assert sum("split-K" in k for k in kern.values()) >= 10, kern
    _cmp_golden(model(case_input(NAME).cuda()), precision)


def test_pipe_split_fp32_dla34():
    name = "b1_480x640_kp"
    model, _, _, _ = dla.build(name, "fp32")
    pred = model(dla34_input(name).cuda())
    dla._cmp(pred, golden(f"dla34_{name}"), dla.TOL["fp32"])


def test_lat_fp32_r18_b1(monkeypatch):
    """The fp32 default: the deep levels on conv_lat<float> (64 x 128 tiles, split-K over
    workgroups), bit-reproducible, within the fp32 tolerance of the golden and of the engine
    without it (TV_LAT_F32=0)."""
    from tauv_vision_amd import engine as E
    img = case_input(NAME).cuda()
    model, _, _, _ = fwd.build(NAME, "fp32")
    kern = _kernels(model, 1)
    assert sum(k.startswith("tv::lat::conv_lat<float>") for k in kern.values()) >= 40, kern
    runs = [model(img) for _ in range(3)]
    for f in ("heatmap", "size", "offset"):
        for r in runs[1:]:
            assert torch.equal(getattr(r, f), getattr(runs[0], f)), f
    _cmp_golden(runs[0], "fp32")
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_LAT_F32": "0"})
    model0, _, _, _ = fwd.build(NAME, "fp32")
    ref = model0(img)
    g = golden(f"model_{NAME}")
    for f in ("heatmap", "size", "offset"):
        scale = max(1.0, float(abs(g[f]).max()))
        d = float((getattr(runs[0], f) - getattr(ref, f)).abs().max())
        assert d <= fwd.TOL["fp32"] * scale, (f, d)


def test_lat_fp32_unsplit_and_b8(monkeypatch):
    """conv_lat<float> without split-K (TV_LAT_SPLIT_F32=1) and on an 8-frame workspace (grouped
    launches of one dependency level)."""
    from tauv_vision_amd import engine as E
    img = case_input(NAME).cuda()
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_LAT_SPLIT_F32": "1"})
    model, _, _, _ = fwd.build(NAME, "fp32")
    _cmp_golden(model(img), "fp32")
    monkeypatch.setattr(E, "_DIAG_KNOBS", {})
    model8, _, _, _ = fwd.build(NAME, "fp32")
    kern = _kernels(model8, 8)
    assert any(k.startswith("tv::lat::conv_lat<float>") for k in kern.values()), kern
    _cmp_golden(model8(torch.cat([torch.flip(img, [-1])] * 7 + [img], 0)), "fp32", 8)
