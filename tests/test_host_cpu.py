"""CPU-only checks: the C-ABI library loads and exports every symbol the header declares,
the native planner reproduces the reference state_dict layout, host-side config logic."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from helpers import models_index, case_by_name, case_state_dict, case_flags

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "tauv_vision_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(tv_\w+)\s*\(", text, re.M)))


def test_library_exports_header_symbols():
    from tauv_vision_amd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib.EXPORTS, f"{s} not bound in _lib.EXPORTS"
    assert L.tv_version().decode().startswith("tauv-vision_amd")


def _desc_for(case, in_h=None, in_w=None, precision="fp32"):
    from tauv_vision_amd.weights import model_desc
    return model_desc(case["heights"], case["channels"], case["downsamples"], models_index()[case["name"]]["head_channels"],
                      in_h or case["in_h"], in_w or case["in_w"], precision)


@pytest.mark.parametrize("name", list(models_index()))
def test_param_layout_matches_reference(name):
    from tauv_vision_amd.weights import param_layout
    case = case_by_name(name)
    got = param_layout(_desc_for(case))
    ref = [(k, tuple(s)) for k, s in models_index()[name]["keys"]]
    assert got == ref


def test_flops_match_survey():
    """"R18" [4,2,2] @480x640 = 197.42 GFLOP/frame; [4,4,8,2,2] = 220.19."""
    from tauv_vision_amd.weights import model_desc, geometry
    g = geometry(model_desc([2] * 5, [128] * 6, 2, [4, 2, 2], 480, 640, "fp16"))
    assert abs(g["flops_per_frame"] / 1e9 - 197.42) < 0.01
    assert (g["out_h"], g["out_w"], g["out_channels"], g["out_cpad"]) == (120, 160, 8, 8)
    g = geometry(model_desc([2] * 5, [128] * 6, 2, [4, 4, 8, 2, 2], 480, 640, "fp16"))
    assert abs(g["flops_per_frame"] / 1e9 - 220.19) < 0.01


@pytest.mark.parametrize("name", list(models_index()))
def test_backbone_only_layout_and_geometry(name):
    """TV_ARCH_CENTERNET_BACKBONE (standalone DLABackbone.forward): exactly the "backbone.*" keys of
    the full network in the same order, output = channels[0] at in / 2^downsamples."""
    from tauv_vision_amd.weights import ARCH_CENTERNET_BACKBONE, model_desc, param_layout, geometry
    case = case_by_name(name)
    full = param_layout(_desc_for(case))
    d = model_desc(case["heights"], case["channels"], case["downsamples"], [1], case["in_h"], case["in_w"],
                   "fp32", arch=ARCH_CENTERNET_BACKBONE)
    assert param_layout(d) == [(k, s) for k, s in full if k.startswith("backbone.")]
    g = geometry(d)
    ds = case["downsamples"]
    assert (g["out_h"], g["out_w"], g["out_channels"], g["out_cpad"]) == (
        case["in_h"] >> ds, case["in_w"] >> ds, case["channels"][0], case["channels"][0])


def test_bad_desc_rejected():
    from tauv_vision_amd.weights import model_desc, geometry
    with pytest.raises(RuntimeError):  # TV_ESHAPE: channels not a multiple of the 16-byte vector
        geometry(model_desc([2], [12, 12], 1, [1], 64, 64, "fp16"))
    with pytest.raises(ValueError):
        model_desc([2], [16], 1, [1])


def test_module_state_dict_layout_and_load():
    import tauv_vision_amd as tv
    case = case_by_name("r18_c16_b2_96x128")
    oc = tv.ObjectConfigSet([tv.ObjectConfig(f"o{i}", tv.AngleConfig(False, None), tv.AngleConfig(False, None),
                                             tv.AngleConfig(False, None), False, False, None) for i in range(4)])
    model = tv.Centernet(tv.DLABackbone(case["heights"], case["channels"], case["downsamples"]), oc)
    keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    assert keys == [(k, tuple(s)) for k, s in models_index()[case["name"]]["keys"]]
    sd = case_state_dict(case["name"])
    v0 = model._version[0]
    res = model.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    assert model._version[0] > v0
    for k, v in model.state_dict().items():
        assert torch.equal(v, sd[k])


def test_config_roundtrip_and_keypoint_index():
    import tauv_vision_amd as tv
    mc = tv.ModelConfig([2] * 5, [128] * 6, 360, 640, 2, 1.0)
    assert tv.ModelConfig.from_dict(mc.to_dict()) == mc
    assert (mc.out_h, mc.out_w, mc.downsample_ratio) == (90, 160, 4)
    A = tv.AngleConfig
    cfgs = [tv.ObjectConfig("a", A(False, 1.0), A(True, 2.0), A(False, None), True, True, [(0, 0, 0), (1, 1, 1)]),
            tv.ObjectConfig("b", A(True, 1.0), A(False, 2.0), A(False, None), False, False, None),
            tv.ObjectConfig("c", A(False, 1.0), A(False, 2.0), A(True, None), False, True, [(2, 2, 2)])]
    s = tv.ObjectConfigSet(cfgs)
    assert s.n_keypoints == 3 and s.n_labels == 3
    assert [s.decode_keypoint_index(i) for i in range(3)] == [(0, 0), (0, 1), (2, 0)]
    assert s.encode_keypoint_index(2, 0) == 2
    s2 = tv.ObjectConfigSet.from_dict(s.to_dict())
    assert s2.to_dict() == s.to_dict()
    assert tv.get_head_channels(s) == [3, 3, 6, 2, 2, 4, 4, 4, 4, 4, 4, 1]
    assert s.get_by_label("c").id == "c"


def test_prediction_field_order_matches_oracle():
    """Pop order of centernet.py:77-90 (roll, pitch, yaw) over heads created yaw, pitch, roll."""
    import oracle
    import tauv_vision_amd as tv
    from tauv_vision_amd.centernet import prediction_from_nhwc
    A = tv.AngleConfig
    oc = tv.ObjectConfigSet([tv.ObjectConfig("a", A(True, 1.0), A(True, 1.0), A(True, 1.0), True, True,
                                             [(0, 0, 0), (1, 1, 1)])])
    hc = tv.get_head_channels(oc)
    H, W = 3, 5
    heads = [torch.randn(2, n, H, W) for n in hc]
    sd = {}
    for i, h in enumerate(heads):  # identity 1x1 "heads" feeding the packing logic of both sides
        pass
    nhwc = torch.cat(heads, 1).permute(0, 2, 3, 1).contiguous()
    ours = prediction_from_nhwc(nhwc, oc)
    # oracle packing from the same head outputs
    flags = dict(keypoints=True, yaw=True, pitch=True, roll=True, depth=True)
    outs = list(heads)

    def nh(t):
        return t.permute(0, 2, 3, 1)
    ref = {"heatmap": outs.pop(0), "keypoint_heatmap": outs.pop(0)}
    t = outs.pop(0)
    ref["keypoint_affinity"] = t.reshape(2, t.shape[1] // 2, 2, H, W)
    ref["size"], ref["offset"] = nh(outs.pop(0)), nh(outs.pop(0))
    for axis in ("roll", "pitch", "yaw"):
        ref[f"{axis}_bin"], ref[f"{axis}_offset"] = nh(outs.pop(0)), nh(outs.pop(0))
    ref["depth"] = nh(outs.pop(0))
    for k, v in ref.items():
        assert torch.equal(getattr(ours, k), v), k
    del flags, sd, oracle


def test_seeded_recipe_matches_golden_recipe():
    from recipe import seeded_state_dict as golden_recipe
    from tauv_vision_amd.weights import seeded_state_dict
    keys = models_index()["dla_var_b1_128x128"]["keys"]
    a = golden_recipe(keys)
    b = seeded_state_dict(keys)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_dla34_param_layout_matches_reference_keys():
    """The native planner's CenterpointDLA34 state_dict layout == the reference module's
    (keys, shapes, order), for both head sets of the goldens; no GPU needed."""
    from helpers import dla34_index
    from tauv_vision_amd.weights import dla34_desc, param_layout, geometry
    for name, e in dla34_index().items():
        d = dla34_desc(e["head_channels"], e["case"]["in_h"], e["case"]["in_w"])
        assert param_layout(d) == [(k, tuple(s)) for k, s in e["keys"]], name
        geo = geometry(d)
        assert (geo["out_h"], geo["out_w"]) == (e["case"]["in_h"] // 4, e["case"]["in_w"] // 4)
        assert geo["out_channels"] == sum(e["head_channels"])


def test_dla34_module_state_dict_loads_reference_checkpoint_keys():
    import tauv_vision_amd as tv
    from helpers import dla34_index, dla34_state_dict
    name = "b2_64x96"
    oc = tv.ObjectConfigSet([tv.ObjectConfig(f"o{i}", tv.AngleConfig(False, 1.0), tv.AngleConfig(False, 1.0),
                                             tv.AngleConfig(False, 1.0), False, False, None) for i in range(4)])
    m = tv.CenterpointDLA34(oc)
    sd = dla34_state_dict(name)
    assert list(m.state_dict().keys()) == list(sd.keys())
    m.load_state_dict(sd)  # strict
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 64, 96)) if not torch.cuda.is_available() else (_ for _ in ()).throw(RuntimeError())
