"""stem_s2.hip: the 7x7 stem (dla.py:150-154, 182-183), block_layers[0].conv1 (3x3 / stride 2,
dla.py:13-19) and the stride-2 stem samples its 1x1 conv_residual reads (dla.py:32-37) in one
launch, the stem output never stored.

The fused launch is the default for the 128-channel "R18" in fp16 / bf16. Checked here:
  * it is the kernel the engine runs (per-op profile names) and the stem op launches nothing;
  * the u8 frame path (LUT staging, both the dword-aligned and the any-width loader) is bit-equal
    to the normalised fp32 NCHW path through the same fused kernel;
  * odd H / W (97 x 129): the last halo row / column past the image, the residual copy and the
    E expansion at the image edge;
  * against the unfused engine (diagnostic knob TV_STEMFUSE=0: stem.hip + conv3x3s2.hip + the
    residual at stride 2 from the stored stem) every Prediction tensor agrees within the
    low-precision tolerance of test_gpu_forward.py (the two differ only in conv1's fp32
    accumulation order), at sizes with partial tiles (Ho % 8, Wo % 32 != 0) and B = 1 / 3;
  * against the reference goldens at 480 x 640 (test_gpu_forward.py's tolerance).
"""
import numpy as np
import pytest
import torch

from helpers import golden, case_input
from recipe import seeded_u8_frames, normalize

import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu

NAME = "r18_c128_b1_480x640"  # seeded production-width weights (any input size)


def _knobs(monkeypatch, knobs):
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", dict(knobs))


def _kernels(model, H, W, B):
    eng = model.engine(torch.device("cuda", 0), H, W)
    frames = torch.zeros((B, H, W, 3), dtype=torch.uint8, device="cuda")
    return {label: k for label, _, _, k in eng.profile(frames, eng.alloc_out(B))}


def _close(a, b, tol, what):
    for f in ("heatmap", "size", "offset"):
        x = getattr(a, f).detach().float().cpu().numpy()
        y = getattr(b, f).detach().float().cpu().numpy()
        scale = max(1.0, float(np.abs(y).max()))
        err = float(np.abs(x - y).max())
        assert err <= tol * scale, f"{what} {f}: {err:.3e} > {tol} * {scale:.3g}"


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("hw,B", [((96, 128), 3), ((96, 126), 1), ((97, 129), 2), ((360, 640), 1)])
def test_fused_matches_unfused(monkeypatch, precision, hw, B):
    H, W = hw
    fr = seeded_u8_frames(B, H, W, seed=H + W)
    img = normalize(fr.permute(0, 3, 1, 2).float() / 255.0).cuda()
    _knobs(monkeypatch, {})
    model, _, _, _ = fwd.build(NAME, precision)
    kern = _kernels(model, H, W, B)
    fused = [k for k in kern.values() if k.startswith("tv::ss2::stem_s2<")]
    assert len(fused) == 1, kern
    assert kern["backbone.dla_down.projection_layer.0"].startswith("(fused into"), kern
    a = model(img)
    b = model.forward_frames(fr.cuda())  # u8: mode 2 when W % 4 == 0, else the byte loader
    for f in ("heatmap", "size", "offset"):
        assert torch.equal(getattr(a, f).cpu(), getattr(b, f).cpu()), f
    _knobs(monkeypatch, {"TV_STEMFUSE": "0"})
    ref_model, _, _, _ = fwd.build(NAME, precision)
    kern_ref = _kernels(ref_model, H, W, B)
    assert not any(k.startswith("tv::ss2::") for k in kern_ref.values()), kern_ref
    _close(a, ref_model(img), fwd.TOL[precision], f"{precision} {hw} B={B}")


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_fused_matches_reference_full_size(monkeypatch, precision):
    _knobs(monkeypatch, {})
    model, _, _, _ = fwd.build(NAME, precision)
    pred = model(case_input(NAME).cuda())
    g = golden(f"model_{NAME}")
    for f in ("heatmap", "size", "offset"):
        ref = g[f]
        got = getattr(pred, f).detach().float().cpu().numpy()
        scale = max(1.0, float(np.abs(ref).max()))
        assert float(np.abs(got - ref).max()) <= fwd.TOL[precision] * scale, f
