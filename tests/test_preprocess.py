"""The node's preprocessing (centernet_node.py:90-92: ToTensor -> Resize((in_h, in_w)) -> Normalize)
on camera frames of another resolution.

The oracle (oracle/ref_preprocess.py) restates torchvision 0.15.2's tensor Resize as torch's
F.interpolate(bilinear, align_corners=False, antialias=False) — torch's own CPU kernel, so the
resize arithmetic is pinned to torch; the torchvision dispatch itself is parity unpinned
(torchvision is absent). Bars: the HIP preprocessing kernel is bit-exact to the oracle; a resized
forward through the fp32 engine is within the north star's 1e-4 of the oracle forward."""
import numpy as np
import pytest
import torch

import oracle
from recipe import normalize, seeded_u8_frames
from test_gpu_forward import build

SIZES = [((480, 640), (360, 640)), ((720, 1280), (360, 640)), ((481, 643), (360, 640)), ((300, 500), (480, 640)),
         ((97, 131), (96, 128)), ((96, 128), (96, 128))]


def test_oracle_identity_resize_is_normalize():
    """Frames already at the model size: Resize is the identity, so preprocessing == the
    ToTensor + Normalize the fused stem path implements (recipe.normalize)."""
    fr = seeded_u8_frames(2, 48, 64, seed=3)
    np.testing.assert_array_equal(oracle.preprocess(fr, 48, 64).numpy(),
                                  normalize(fr.permute(0, 3, 1, 2).float() / 255.0).numpy())


def test_oracle_resize_matches_torch_bilinear():
    fr = seeded_u8_frames(1, 37, 53, seed=4)
    img = fr.permute(0, 3, 1, 2).float() / 255.0
    ref = torch.nn.functional.interpolate(img, (20, 30), mode="bilinear", align_corners=False)
    np.testing.assert_array_equal(oracle.preprocess(fr, 20, 30).numpy(), normalize(ref).numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", SIZES)
def test_gpu_preprocess_bit_exact(src, dst):
    import tauv_vision_amd as tv
    fr = seeded_u8_frames(2, src[0], src[1], seed=src[0] + dst[0])
    got = tv.preprocess(fr.cuda(), dst[0], dst[1]).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.preprocess(fr, dst[0], dst[1]).numpy())


@pytest.mark.gpu
def test_gpu_forward_frames_resized():
    """480x640 camera frames into the 360x640 torpedo-geometry model (samples_torpedo.py:4-6)."""
    import tauv_vision_amd as tv
    model, oc, mc, case = build("torpedo_c16_b1_360x640", "fp32")
    fr = seeded_u8_frames(2, 480, 640, seed=77)
    pred = model.forward_frames(fr.cuda(), (360, 640))
    from helpers import case_state_dict, case_flags
    with torch.no_grad():
        ref = oracle.centernet_forward(case_state_dict("torpedo_c16_b1_360x640"), oracle.preprocess(fr, 360, 640),
                                       case["heights"], case["downsamples"], case_flags(case))
    for f in ("heatmap", "size", "offset"):
        a, b = getattr(pred, f).cpu().numpy(), getattr(ref, f).numpy()
        assert a.shape == b.shape
        assert float(np.abs(a - b).max()) <= 1e-4 * max(1.0, float(np.abs(b).max())), f
    # detect() resizes to model_config's size like the node
    dets = model.detect(fr.cuda(), mc, 20, 0.05)
    want = tv.decode(pred, mc, 20, 0.05)
    assert [[(int(d.label), float(d.score)) for d in b] for b in dets] == \
        [[(int(d.label), float(d.score)) for d in b] for b in want]
