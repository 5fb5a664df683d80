"""conv_lat.hip (the small-level latency kernel: small tiles, K split over the waves of a
workgroup) against the reference goldens.

By default the engine picks conv_lat only for layers its other kernels spread over fewer work
units than there are CUs (the deep DLA levels). These tests force it onto every eligible layer
(diagnostic knob TV_LAT_UNITS huge, the one-shot conv_burst.hip off: TV_BURST=0) at B = 1 and 3,
so 3x3 / stride-2 / Root concatenations / the fused 1x1 residual / DLA-34's identity residuals all
run through it at full size, and compare with the reference outputs at the same tolerances as the
default path (test_gpu_forward.py, test_gpu_dla34.py). By default conv_burst.hip takes the conv_lat
layers it represents (tests/test_gpu_conv_burst.py); conv_lat keeps the strided 3x3 ones and the
wide DLA-34 levels.
"""
import pytest
import torch

from helpers import golden, case_input, dla34_input

import test_gpu_dla34 as dla
import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu


def _force(monkeypatch):
    """Engines built in this test get the diagnostic knob TV_LAT_UNITS (tv_engine_create_diag);
    the product path reads no environment."""
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_LAT_UNITS": str(10 ** 9), "TV_BURST": "0"})


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("B", [1, 3])
def test_lat_everywhere_r18_full_size(monkeypatch, precision, B):
    _force(monkeypatch)
    name = "r18_c128_b1_480x640"
    model, oc, mc, case = fwd.build(name, precision)
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    frames = torch.zeros((B, 480, 640, 3), dtype=torch.uint8, device="cuda")
    kern = {label: k for label, _, _, k in eng.profile(frames, eng.alloc_out(B))}
    n_lat = sum(k.startswith("tv::lat::conv_lat<") for k in kern.values())
    assert n_lat >= 60, kern  # every 128-channel conv but the stem and the fused heads
    img = case_input(name).cuda()
    # the golden frame at the last batch position (M not a multiple of the 64-pixel tile)
    pred = model(torch.cat([torch.flip(img, [-1])] * (B - 1) + [img], 0))
    g = golden(f"model_{name}")
    for f in ("heatmap", "size", "offset"):
        ref = g[f]
        got = getattr(pred, f)[B - 1:].detach().cpu().numpy()
        scale = max(1.0, float(abs(ref).max()))
        assert float(abs(got - ref).max()) <= fwd.TOL[precision] * scale, f


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_lat_everywhere_dla34(monkeypatch, precision):
    _force(monkeypatch)
    name = "b1_480x640_kp"
    model, oc, mc, case = dla.build(name, precision)
    pred = model(dla34_input(name).cuda())
    dla._cmp(pred, golden(f"dla34_{name}"), dla.TOL[precision])


def test_lat_default_selection_b32():
    """At the bench's 32-frame slice the deep levels (15x20 and below) leave the halo kernels: the
    stride-1 layers whose tiles fit one round for the one-shot conv_burst, the rest for conv_lat; the 120x160 /
    60x80 levels stay on the halo kernels."""
    name = "r18_c128_b1_480x640"
    model, oc, mc, case = fwd.build(name, "fp16")
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    frames = torch.zeros((32, 480, 640, 3), dtype=torch.uint8, device="cuda")
    kern = {label: k for label, _, _, k in eng.profile(frames, eng.alloc_out(32))}
    assert kern["backbone.dla_down.tree_layers.2.tree_l.tree_r.conv2+conv_residual"].startswith("tv::lat::conv_lat<"), kern
    assert kern["backbone.dla_down.tree_layers.4.tree_r.root.conv"].startswith("tv::burst::conv_burst<"), kern
    assert kern["backbone.dla_down.tree_layers.2.tree_l.tree_l.conv1"].startswith("tv::lat::conv_lat<"), kern
    assert kern["backbone.dla_down.tree_layers.0.tree_l.tree_r.conv1"].startswith("tv::c3::conv3x3<"), kern
    assert kern["backbone.multi_ida_up.ida_up_layers.0.output_layers.0.0"].startswith("tv::c3::conv3x3<"), kern


def test_lat_split_k_b1(monkeypatch):
    """At B=1 the conv_lat layers can run split-K over workgroups (several workgroups per tile, the
    last to arrive sums the fp32 partial tiles in slice order; by default only layers of >= 32
    k-steps, so here forced for R18's 18-20 k-step layers with TV_LAT_SPLIT_MIN=0): repeated forwards
    are bit-identical whichever workgroup arrives last, and the result matches the unsplit kernel
    (knob TV_LAT_SPLIT=1) within the fp16 tolerance of the golden comparison."""
    from tauv_vision_amd import engine as E
    name = "r18_c128_b1_480x640"
    img = case_input(name).cuda()
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_BURST": "0", "TV_LAT_SPLIT_MIN": "0"})  # every deep layer on conv_lat, split
    model, oc, mc, case = fwd.build(name, "fp16")
    runs = [model(img) for _ in range(3)]
    for f in ("heatmap", "size", "offset"):
        for r in runs[1:]:
            assert torch.equal(getattr(r, f), getattr(runs[0], f)), f
    monkeypatch.setattr(E, "_DIAG_KNOBS", {"TV_LAT_SPLIT": "1", "TV_BURST": "0"})
    model1, _, _, _ = fwd.build(name, "fp16")
    ref = model1(img)
    g = golden(f"model_{name}")
    for f in ("heatmap", "size", "offset"):
        scale = max(1.0, float(abs(g[f]).max()))
        d = float((getattr(runs[0], f) - getattr(ref, f)).abs().max())
        assert d <= fwd.TOL["fp16"] * scale, (f, d)
        got = getattr(runs[0], f).detach().cpu().numpy()
        assert float(abs(got - g[f]).max()) <= fwd.TOL["fp16"] * scale, f
