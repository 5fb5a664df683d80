"""The engine's latency-path schedule (engine.cpp make_workspace): on workspaces of <= 8 frames
the ops run by dependency level — the MultiIDAUp wavefront, the IDAUpReverse projections early
(dla.py:265-284, 340-357, 377-390) — and the conv_lat layers / ConvTranspose up-steps of one level
share a launch (conv_lat.hip conv_lat_group, convt.hip convt_add_group), the arena's lifetimes
counted in levels. The same kernels run on the same data in another launch order, so every
output must be bit-identical to the plan-order execution (diagnostic knob TV_LATGROUP=0), at
B = 1 and 3 (R18, DLA-34) and for the protonet's ConvTranspose phase GEMMs; profile() runs the
schedule's order one op per launch and must agree as well. B = 8 is the largest grouped workspace
(grouped conv_lat / convt launches at their CU packing limits) and B = 16 runs as two concurrent
8-frame slices, each on its own grouped schedule."""
import numpy as np
import pytest
import torch

from helpers import case_input, dla34_input
from recipe import seeded_u8_frames, normalize

import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu


def _knobs(monkeypatch, knobs):
    from tauv_vision_amd import engine as E
    monkeypatch.setattr(E, "_DIAG_KNOBS", dict(knobs))


def _fields(pred):
    return {f: getattr(pred, f).detach().cpu() for f in fwd.FIELDS if getattr(pred, f) is not None}


@pytest.mark.parametrize("name,B", [("r18_c128_b1_480x640", 1), ("r18_c128_b1_480x640", 3),
                                    ("r18_c128_b1_480x640", 8), ("r18_c128_b1_480x640", 16),
                                    ("dla34:b1_480x640_kp", 1)])
@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_grouped_schedule_is_bit_identical(monkeypatch, name, B, precision):
    if name.startswith("dla34:"):
        name = name.split(":", 1)[1]
        import test_gpu_dla34 as dla
        builder = lambda: dla.build(name, precision)[0]  # noqa: E731
        x = dla34_input(name)
    else:
        builder = lambda: fwd.build(name, precision)[0]  # noqa: E731
        x = case_input(name)
    H, W = x.shape[-2:]
    if B > 1:
        x = normalize(seeded_u8_frames(B, H, W, seed=B).permute(0, 3, 1, 2).float() / 255.0)
    x = x.cuda()
    _knobs(monkeypatch, {})
    a = _fields(builder()(x))
    _knobs(monkeypatch, {"TV_LATGROUP": "0"})
    b = _fields(builder()(x))
    assert a.keys() == b.keys()
    for f in a:
        assert torch.equal(a[f], b[f]), f"{name} B={B} {precision} {f}"


def test_profile_runs_the_schedule(monkeypatch):
    """profile() (one op per launch, in the schedule's order) writes the same output as the
    grouped forward, and reports every op once."""
    _knobs(monkeypatch, {})
    model, _, _, _ = fwd.build("r18_c128_b1_480x640", "fp16")
    H, W = 480, 640
    fr = seeded_u8_frames(1, H, W, seed=7).cuda()
    eng = model.engine(torch.device("cuda", 0), H, W)
    out_a = eng.alloc_out(1)
    eng.forward_u8(fr, out_a)
    out_b = eng.alloc_out(1)
    ops = eng.profile(fr, out_b)
    torch.cuda.synchronize()
    assert len(ops) == len({o[0] for o in ops})
    assert torch.equal(out_a, out_b)


def test_protonet_grouped_schedule_is_bit_identical(monkeypatch):
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    from recipe import protonet_case, protonet_inputs
    from test_yolact import SCALES, VAR
    c = protonet_case("protonet_f64_k16_b1_9x17")
    sd, _ = protonet_inputs(c)
    x = torch.randn(3, 64, 9, 17, generator=torch.Generator().manual_seed(5)).cuda()
    outs = []
    for knobs in ({}, {"TV_LATGROUP": "0"}):
        _knobs(monkeypatch, knobs)
        m = Masknet(YolactConfig(640, 360, SCALES, (1,), VAR, feature_depth=64, n_prototype_masks=16),
                    precision="fp16")
        m.load_state_dict(sd)
        outs.append(m(x).cpu().numpy())
    np.testing.assert_array_equal(outs[0], outs[1])
