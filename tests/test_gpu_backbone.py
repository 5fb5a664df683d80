"""DLABackbone.forward on its own (reference dla.py:393-416): the backbone-only native plan
(TV_ARCH_CENTERNET_BACKBONE) against the oracle's backbone (oracle.backbone_forward, the
restatement the whole-network goldens pin), on the seeded weights / inputs of the golden cases.
fp32 parity mode within 1e-4 x max(1, |ref|max); fp16 / bf16 within the whole-network
tolerances of test_gpu_forward.py."""
import numpy as np
import pytest
import torch

import oracle
from helpers import case_by_name, case_state_dict, case_input

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-4, "fp16": 2e-3, "bf16": 1.5e-2}


def _backbone(name, precision):
    import tauv_vision_amd as tv
    case = case_by_name(name)
    bb = tv.DLABackbone(case["heights"], case["channels"], case["downsamples"], precision=precision)
    sd = case_state_dict(name)
    bb.load_state_dict({k[len("backbone."):]: v for k, v in sd.items() if k.startswith("backbone.")})
    return bb.cuda().eval(), case, sd


@pytest.mark.parametrize("name,precision", [("r18_c16_b2_96x128", "fp32"), ("square_c32_b2_128", "fp32"),
                                            ("r18_c128_b1_480x640", "fp32"), ("r18_c128_b1_480x640", "fp16"),
                                            ("r18_c128_b1_480x640", "bf16")])
def test_backbone_forward_matches_oracle(name, precision):
    bb, case, sd = _backbone(name, precision)
    img = case_input(name)
    got = bb(img.cuda())
    with torch.no_grad():
        ref = oracle.backbone_forward(sd, img, case["heights"], case["downsamples"])
    assert tuple(got.shape) == tuple(ref.shape) == (img.shape[0], case["channels"][0],
                                                    img.shape[2] >> case["downsamples"],
                                                    img.shape[3] >> case["downsamples"])
    scale = max(1.0, float(ref.abs().max()))
    err = float((got.cpu() - ref).abs().max())
    assert err <= TOL[precision] * scale, f"{err:.3e} > {TOL[precision]} x {scale:.3g}"


def test_backbone_inside_centernet_unchanged():
    """The standalone backbone and Centernet(backbone, ...) share the parameters: a Centernet
    built around the backbone still matches its golden heads output."""
    import test_gpu_forward as fwd
    from helpers import golden
    name = "r18_c16_b2_96x128"
    model, oc, mc, case = fwd.build(name, "fp32")
    img = case_input(name).cuda()
    feat = model.backbone(img)
    assert feat.shape[1] == case["channels"][0]
    fwd._cmp(model(img), golden(f"model_{name}"), fwd.TOL["fp32"])
