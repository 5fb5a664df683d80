"""Training targets (reference loss.py:31-135): the oracle restatement against
the reference's own outputs (tests/golden/targets_*.npz, made by gen_golden_targets.py), and the
HIP kernels (tv_train_heatmap / tv_train_keypoint_targets through tauv_vision_amd.loss) against
both. The Gaussians are fp32 exp of fp32 arguments formed exactly as the reference forms them:
the GPU exp may differ from torch's CPU exp by an ulp, so those planes are compared at 2e-7
absolute (values in [0, 1]). The affinity vectors are d / sqrt(d0^2 + d1^2): the reference's
torch.sqrt on CPU is MKL VML's vsSqrt, which is not correctly rounded (measured here: 0.6% of
fp32 results one ulp below the correctly rounded root, never above), while the kernel's sqrt
and quotient are correctly rounded, so those planes are also compared at 2e-7 (values in
[-1, 1]; a differently chosen winning instance would show as an O(1) error)."""
import types

import numpy as np
import pytest
import torch

from helpers import golden
from oracle import ref_targets as rt

CASES = ["targets_b2_o5_l3_240x320", "targets_b3_o9_l4_480x640", "targets_b2_o4_l2_96x128_tinysigma"]


def _truth(g):
    t = lambda k: torch.from_numpy(g[k])  # noqa: E731
    return types.SimpleNamespace(valid=t("valid"), label=t("label"), center=t("center"),
                                 keypoint_valid=t("keypoint_valid"), keypoint_label=t("keypoint_label"),
                                 keypoint_center=t("keypoint_center"),
                                 keypoint_object_index=t("keypoint_object_index"))


def _configs(g):
    import tauv_vision_amd as tv
    mc = tv.ModelConfig([2] * 5, [16] * 6, int(g["in_h"]), int(g["in_w"]), int(g["downsamples"]), 1.0)
    tc = types.SimpleNamespace(keypoint_heatmap_sigma=float(g["keypoint_heatmap_sigma"]),
                               keypoint_affinity_sigma=float(g["keypoint_affinity_sigma"]))
    return mc, tc


@pytest.mark.parametrize("name", CASES)
def test_oracle_targets_match_reference(name):
    g = golden(name)
    mc, tc = _configs(g)
    truth = _truth(g)
    heat = rt.generate_heatmap(truth, mc, tc, int(g["n_labels"]))
    np.testing.assert_array_equal(heat.numpy(), g["heatmap"])
    kh, kaw, kaff = rt.generate_keypoint_heatmap(truth, mc, tc, int(g["n_keypoints"]))
    np.testing.assert_array_equal(kh.numpy(), g["keypoint_heatmap"])
    np.testing.assert_array_equal(kaw.numpy(), g["keypoint_affinity_weight"])
    np.testing.assert_array_equal(kaff.numpy(), g["keypoint_affinity"])
    np.testing.assert_array_equal(rt.out_index_for_position(truth.center, mc).numpy(), g["out_index"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_targets_match_reference(name):
    from tauv_vision_amd import loss as L
    g = golden(name)
    mc, tc = _configs(g)
    t = lambda k: torch.from_numpy(g[k]).cuda()  # noqa: E731
    truth = L.PoseSample(valid=t("valid"), label=t("label"), center=t("center"), keypoint_valid=t("keypoint_valid"),
                         keypoint_label=t("keypoint_label"), keypoint_center=t("keypoint_center"),
                         keypoint_object_index=t("keypoint_object_index"))
    oc = types.SimpleNamespace(n_labels=int(g["n_labels"]), n_keypoints=int(g["n_keypoints"]))
    heat = L.generate_heatmap(truth, mc, tc, oc)
    assert heat.is_cuda and heat.dtype == torch.float32
    np.testing.assert_allclose(heat.cpu().numpy(), g["heatmap"], rtol=0, atol=2e-7)
    kh, kaw, kaff = L.generate_keypoint_heatmap(truth, mc, tc, oc)
    np.testing.assert_allclose(kh.cpu().numpy(), g["keypoint_heatmap"], rtol=0, atol=2e-7)
    np.testing.assert_allclose(kaw.cpu().numpy(), g["keypoint_affinity_weight"], rtol=0, atol=2e-7)
    np.testing.assert_allclose(kaff.cpu().numpy(), g["keypoint_affinity"], rtol=0, atol=2e-7)
    # the Gaussian peaks (value 1 exactly at the center cell) land on the same cells
    np.testing.assert_array_equal(heat.cpu().numpy() == 1.0, g["heatmap"] == 1.0)
    np.testing.assert_array_equal(L.out_index_for_position(truth.center, mc).cpu().numpy(), g["out_index"])


# One element behind the 2e-7 tolerance above (float32 bits 0x3fee9794 = 1.8640008): torch's CPU
# sqrt (MKL VML on this image, AVX512) returns 1.3652841, one ulp below the correctly rounded root
# 1.3652842 (the float64 root rounded to float32, exact for float32 inputs). The kernel's sqrt is
# correctly rounded, so the affinity planes can differ from the reference's by that ulp.
SQRT_X_BITS = 0x3FEE9794


def _f32(bits):
    return np.array([bits], dtype=np.uint32).view(np.float32)


def test_torch_cpu_sqrt_within_one_ulp_below():
    x = _f32(SQRT_X_BITS)
    cr = np.sqrt(x.astype(np.float64)).astype(np.float32)
    assert cr.view(np.uint32)[0] == 0x3FAEC1A2  # 1.3652842
    got = torch.sqrt(torch.from_numpy(x)).numpy()
    # correctly rounded, or (MKL VML) exactly one ulp below — never above, never further
    assert int(cr.view(np.int32)[0]) - int(got.view(np.int32)[0]) in (0, 1)
    # the same bound over a million uniform samples in [0, 2): the tolerance's premise
    xs = (torch.rand(1 << 20, generator=torch.Generator().manual_seed(0)) * 2).numpy()
    d = np.sqrt(xs.astype(np.float64)).astype(np.float32).view(np.int32).astype(np.int64) - \
        torch.sqrt(torch.from_numpy(xs)).numpy().view(np.int32).astype(np.int64)
    assert d.min() >= 0 and d.max() <= 1


def test_targets_reject_inconsistent_out_shape():
    """The kernels derive out_h / out_w from in_h // downsample_ratio: a config that disagrees is
    refused before anything is launched (a duck-typed config would otherwise be written OOB)."""
    from tauv_vision_amd import loss as L
    mc = types.SimpleNamespace(in_h=64, in_w=96, downsample_ratio=4, out_h=16, out_w=25)
    tc = types.SimpleNamespace(keypoint_heatmap_sigma=2.0, keypoint_affinity_sigma=3.0)
    oc = types.SimpleNamespace(n_labels=2, n_keypoints=2)
    truth = types.SimpleNamespace(valid=torch.zeros(1, 0, dtype=torch.bool))
    with pytest.raises(ValueError, match="out_h/out_w"):
        L.generate_heatmap(truth, mc, tc, oc)
    with pytest.raises(ValueError, match="out_h/out_w"):
        L.generate_keypoint_heatmap(truth, mc, tc, oc)


@pytest.mark.gpu
def test_gpu_targets_empty_and_all_invalid():
    from tauv_vision_amd import loss as L
    import tauv_vision_amd as tv
    mc = tv.ModelConfig([2] * 5, [16] * 6, 64, 96, 1, 1.0)
    tc = types.SimpleNamespace(keypoint_heatmap_sigma=2.0, keypoint_affinity_sigma=3.0)
    oc = types.SimpleNamespace(n_labels=2, n_keypoints=2)
    z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device="cuda")  # noqa: E731
    for n in (0, 3):  # no objects at all / every object and instance invalid
        truth = L.PoseSample(valid=z(2, n, dt=torch.bool), label=z(2, n, dt=torch.int64), center=z(2, n, 2),
                             keypoint_valid=z(2, n, dt=torch.bool), keypoint_label=z(2, n, dt=torch.int64),
                             keypoint_center=z(2, n, 2), keypoint_object_index=z(2, n, dt=torch.int64))
        assert float(L.generate_heatmap(truth, mc, tc, oc).abs().sum()) == 0.0
        kh, kaw, kaff = L.generate_keypoint_heatmap(truth, mc, tc, oc)
        assert float(kh.abs().sum() + kaw.abs().sum() + kaff.abs().sum()) == 0.0
