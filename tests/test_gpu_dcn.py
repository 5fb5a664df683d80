"""DCNv2 kernels driven directly (tv_diag_dcn_conv), pinned to identities of the reference's
DeformConv (centerpoint_dla.py:360-392: torchvision DeformConv2d(x, offset, sigmoid(mask)),
3x3 / stride 1 / pad 1). torchvision is absent, so the general bilinear case is "parity
unpinned" (checked only against the oracle restatement, oracle/ref_dla34.py:35); these
identities need no torchvision:
  * zero offsets + unit mask          == conv2d(x, W, padding=1)   (F.conv2d, fp32 CPU)
  * integer offsets (per tap) + unit mask == the 3x3 conv whose tap k reads x shifted by
                                         offset k, zeros outside the image (computed here)
  * offsets past the image            == bias (every sample is 0)
Inputs and weights are rounded to the compute dtype first, so in the identities the only
difference left is fp32 accumulation order and the output rounding. Variants: 0 dcn_gemm,
1 dcn_gemm64, 2 dcn_gemm64 with 64-pixel tiles (same blend arithmetic and K order: bit-equal),
3 the unfused path (sampling into a column tensor + the implicit-GEMM conv kernel; fp32's path),
4 dcn_win (C == N == 64: the tile's input window staged in LDS, corners outside it gathered from
global memory; same arithmetic and K order as dcn_gemm64: bit-equal to it — the bilinear case's
offsets of sigma 2.5 exercise the out-of-window path).
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle.ref_dla34 import deform_conv2d

pytestmark = pytest.mark.gpu

DT = {"fp32": (torch.float32, 0), "fp16": (torch.float16, 1), "bf16": (torch.bfloat16, 2)}
# output rounding of the compute dtype (relative), for the identities
ULP = {"fp32": 2e-6, "fp16": 1.0e-3, "bf16": 8.0e-3}
# general bilinear case vs the oracle: the sampled column values are rounded to the compute dtype
# before the MFMA (the oracle keeps them fp32)
TOL = {"fp32": 2e-5, "fp16": 4e-3, "bf16": 3e-2}


def variants(precision, C, N=None):
    if precision == "fp32":
        return [3]
    v = [0, 1, 2, 3, 5, 6, 7, 8] if C % 64 == 0 else [0, 3]
    return v + [4] if C == 64 and N == 64 else v


def dcn_gpu(x, om, w, b, act, precision, variant):
    """x [B,C,H,W], om [B,27,H,W] (dy,dx per tap + mask logits), already rounded; -> [B,N,H,W] fp32."""
    from tauv_vision_amd import _lib
    dt, code = DT[precision]
    B, C, H, W = x.shape
    N = w.shape[0]
    xd = x.permute(0, 2, 3, 1).to(dt).cuda().contiguous()
    omp = torch.zeros(B, H, W, 32)
    omp[..., :27] = om.permute(0, 2, 3, 1)
    omd = omp.to(dt).cuda().contiguous()
    out = torch.full((B, H, W, N), float("nan"), dtype=dt, device="cuda")
    wc, bc = w.float().contiguous(), b.float().contiguous()
    L = _lib.lib()
    _lib.check(L.tv_diag_dcn_conv(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(omd.data_ptr()), B, H, W, C, 32,
                                  ctypes.c_void_p(wc.data_ptr()), ctypes.c_void_p(bc.data_ptr()), N, act, code, variant,
                                  ctypes.c_void_p(out.data_ptr()), _lib.stream_of(out.device)), "dcn")
    return out.float().cpu().permute(0, 3, 1, 2)


def rnd(t, precision):
    return t.to(DT[precision][0]).float()


def inputs(B, C, H, W, N, precision, seed):
    g = torch.Generator().manual_seed(seed)
    x = rnd(torch.randn(B, C, H, W, generator=g), precision)
    w = rnd(torch.randn(N, C, 3, 3, generator=g) / (3.0 * C ** 0.5), precision)
    b = torch.randn(N, generator=g) * 0.1
    return x, w, b, g


def om_of(dy, dx, logit):
    """[B,27,H,W]: channel 2k = dy of tap k, 2k+1 = dx, 18+k = mask logit."""
    return torch.cat([torch.stack([dy, dx], 2).flatten(1, 2), logit], 1)


def assert_close(got, ref, rel, what):
    scale = float(ref.abs().max()) + 1e-6
    err = float((got - ref).abs().max())
    assert err <= rel * scale, f"{what}: max err {err:.3g} > {rel:.3g} x {scale:.3g}"


SHAPES = [(2, 64, 13, 19, 64), (1, 128, 9, 24, 128), (2, 32, 7, 11, 64), (1, 256, 5, 7, 128)]


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("shape", SHAPES)
def test_dcn_zero_offsets_unit_mask_is_conv(precision, shape):
    B, C, H, W, N = shape
    x, w, b, _ = inputs(B, C, H, W, N, precision, 11)
    zero = torch.zeros(B, 9, H, W)
    om = rnd(om_of(zero, zero, torch.full((B, 9, H, W), 30.0)), precision)  # sigmoid(30) == 1.0f
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    outs = {v: dcn_gpu(x, om, w, b, 0, precision, v) for v in variants(precision, C, N)}
    for v, o in outs.items():
        assert_close(o, ref, ULP[precision], f"variant {v}")
    fused = [o for v, o in outs.items() if v in (0, 1, 2, 4, 5)]
    for o in fused[1:]:
        assert torch.equal(o, fused[0]), "dcn_gemm / dcn_gemm64 / dcn_win / dcn_gemm64d tilings must be bit-identical"


def shifted_conv(x, w, b, dy, dx):
    """3x3 conv whose tap k = (i, j) reads x[y + i - 1 + dy[k], x + j - 1 + dx[k]] (0 outside)."""
    B, C, H, W = x.shape
    P = 8
    xp = F.pad(x.double(), (P, P, P, P))
    out = torch.zeros(B, w.shape[0], H, W, dtype=torch.float64) + b.double().view(1, -1, 1, 1)
    for k in range(9):
        i, j = divmod(k, 3)
        sy, sx = P + i - 1 + int(dy[k]), P + j - 1 + int(dx[k])
        win = xp[:, :, sy:sy + H, sx:sx + W]
        out += torch.einsum("nc,bchw->bnhw", w[:, :, i, j].double(), win)
    return out.float()


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("shape", SHAPES[:3])
def test_dcn_integer_offsets_is_shifted_conv(precision, shape):
    B, C, H, W, N = shape
    x, w, b, g = inputs(B, C, H, W, N, precision, 12)
    dy = torch.randint(-3, 4, (9,), generator=g)
    dx = torch.randint(-3, 4, (9,), generator=g)
    om = om_of(dy.float().view(1, 9, 1, 1).expand(B, 9, H, W), dx.float().view(1, 9, 1, 1).expand(B, 9, H, W),
               torch.full((B, 9, H, W), 30.0))
    om = rnd(om, precision)
    ref = shifted_conv(x, w, b, dy, dx)
    for v in variants(precision, C, N):
        assert_close(dcn_gpu(x, om, w, b, 0, precision, v), ref, ULP[precision], f"variant {v}")


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
def test_dcn_offsets_outside_image_give_bias(precision):
    B, C, H, W, N = 1, 64, 6, 10, 64
    x, w, b, g = inputs(B, C, H, W, N, precision, 13)
    far = torch.full((B, 9, H, W), 1000.0)
    for sgn in (1.0, -1.0):
        om = rnd(om_of(sgn * far, far, torch.randn(B, 9, H, W, generator=g)), precision)
        want = rnd(b.view(1, N, 1, 1).expand(B, N, H, W), precision)
        for v in variants(precision, C, N):
            got = dcn_gpu(x, om, w, b, 0, precision, v)
            assert torch.equal(got, want), f"variant {v}: samples outside the image must be 0"
        relu = dcn_gpu(x, om, w, b, 1, precision, variants(precision, C)[0])
        assert torch.equal(relu, want.clamp_min(0.0))


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("shape", SHAPES)
def test_dcn_bilinear_vs_oracle_restatement(precision, shape):
    """General case (fractional offsets reaching past the borders, random masks) against the
    restated torchvision algorithm — parity unpinned (no torchvision, no reference fixture)."""
    B, C, H, W, N = shape
    x, w, b, g = inputs(B, C, H, W, N, precision, 14)
    om = rnd(om_of(torch.randn(B, 9, H, W, generator=g) * 2.5, torch.randn(B, 9, H, W, generator=g) * 2.5,
                   torch.randn(B, 9, H, W, generator=g) * 2.0), precision)
    off, logit = om[:, :18], om[:, 18:]
    ref = deform_conv2d(x.double(), off.double(), torch.sigmoid(logit.double()), w.double(), b.double()).float()
    outs = {v: dcn_gpu(x, om, w, b, 1, precision, v) for v in variants(precision, C, N)}
    for v, o in outs.items():
        assert_close(o, ref.clamp_min(0.0), TOL[precision], f"variant {v}")
    fused = [o for v, o in outs.items() if v in (0, 1, 2, 4, 5)]
    for o in fused[1:]:
        assert torch.equal(o, fused[0]), "dcn_gemm / dcn_gemm64 / dcn_win / dcn_gemm64d tilings must be bit-identical"


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("sigma", [0.7, 4.0])
def test_dcn_window_kernel_multi_tile_bit_equal(precision, sigma):
    """dcn_win over several 16 x 16 tiles per frame (partial tiles at the right and bottom edges, the
    persistent tile loop, the next tile's window staged under the last tap) with offsets mostly inside
    the window (sigma 0.7) or mostly past it (sigma 4): bit-equal to dcn_gemm64, close to the
    restated torchvision algorithm."""
    B, C, H, W, N = 3, 64, 37, 45, 64
    x, w, b, g = inputs(B, C, H, W, N, precision, 21)
    om = rnd(om_of(torch.randn(B, 9, H, W, generator=g) * sigma, torch.randn(B, 9, H, W, generator=g) * sigma,
                   torch.randn(B, 9, H, W, generator=g) * 2.0), precision)
    got = dcn_gpu(x, om, w, b, 1, precision, 4)
    assert torch.equal(got, dcn_gpu(x, om, w, b, 1, precision, 1)), "dcn_win must equal dcn_gemm64 bit for bit"
    off, logit = om[:, :18], om[:, 18:]
    ref = deform_conv2d(x.double(), off.double(), torch.sigmoid(logit.double()), w.double(), b.double()).float()
    assert_close(got, ref.clamp_min(0.0), TOL[precision], "dcn_win")


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("shape", [(3, 64, 37, 45, 64), (2, 128, 30, 41, 128), (1, 256, 15, 20, 128), (4, 64, 60, 80, 64)])
def test_dcn_deep_prefetch_bit_equal(precision, shape):
    """dcn_gemm64d (variant 5: gathers two k-steps ahead, sampling state three taps ahead in a
    4-slot ring, every main-loop load unconditional) over many workgroups, odd step counts (9 k-steps
    at C = 64) and 2 / 4 channel blocks per tap: bit-equal to dcn_gemm64 on 64-pixel tiles."""
    B, C, H, W, N = shape
    x, w, b, g = inputs(B, C, H, W, N, precision, 23)
    om = rnd(om_of(torch.randn(B, 9, H, W, generator=g) * 1.5, torch.randn(B, 9, H, W, generator=g) * 1.5,
                   torch.randn(B, 9, H, W, generator=g) * 2.0), precision)
    got = dcn_gpu(x, om, w, b, 1, precision, 5)
    assert torch.equal(got, dcn_gpu(x, om, w, b, 1, precision, 2)), "dcn_gemm64d must equal dcn_gemm64 bit for bit"


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("shape", [(1, 256, 30, 40, 256), (1, 64, 60, 80, 64), (2, 128, 15, 21, 128), (1, 256, 5, 7, 128)])
def test_dcn_split_k(precision, shape):
    """dcn_gemm64 split-K over tap ranges (variants 6 / 7 / 8: 3 / 4 / 9 slices of the 9 taps — the
    engine's form for DLA-34's small-batch DeformConvs): each slice's fp32 partial accumulators go
    through the slab and the last-arriving workgroup sums them in slice order, so the result is
    the unsplit kernel's up to the fp32 summation order (within the output rounding) and
    bit-identical run to run; the tickets reset themselves (the repeats reuse fresh slabs here, the
    engine's workspace reuse is covered by the DLA-34 B=1 tests)."""
    B, C, H, W, N = shape
    x, w, b, g = inputs(B, C, H, W, N, precision, 29)
    om = rnd(om_of(torch.randn(B, 9, H, W, generator=g) * 1.5, torch.randn(B, 9, H, W, generator=g) * 1.5,
                   torch.randn(B, 9, H, W, generator=g) * 2.0), precision)
    ref = dcn_gpu(x, om, w, b, 1, precision, 2)
    for v in (6, 7, 8):
        got = dcn_gpu(x, om, w, b, 1, precision, v)
        assert torch.isfinite(got).all(), f"variant {v}"
        assert torch.equal(got, dcn_gpu(x, om, w, b, 1, precision, v)), f"variant {v}: not deterministic"
        assert_close(got, ref, ULP[precision], f"variant {v} vs unsplit")
