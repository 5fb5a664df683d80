"""tv_engine_forward_insitu[_u8] (the bench's in-situ roofline timing): one forward exactly as the
timed region runs it — concurrent slices, grouped launches — with an event before each launch on
its slice's stream. Its output must equal the plain forward's bit for bit, every slice must report
a positive time for every launching op, and the per-slice launch times must sum to about the
forward's wall time (they tile each slice's stream)."""
import pytest
import torch

import test_gpu_forward as fwd

pytestmark = pytest.mark.gpu

NAME = "r18_c128_b1_480x640"


@pytest.mark.parametrize("B", [1, 20])
def test_insitu_forward_matches_forward(B):
    model, _, _, _ = fwd.build(NAME, "fp16")
    eng = model.engine(torch.device("cuda", 0), 480, 640)
    g = torch.Generator().manual_seed(5)
    frames = torch.randint(0, 256, (B, 480, 640, 3), generator=g, dtype=torch.uint8).cuda()
    ref = eng.forward_u8(frames)
    rows = eng.profile(frames[:eng.slices(B)[0]].contiguous())
    out = eng.alloc_out(B)
    sl = eng.profile_insitu(frames, out, cap=len(rows))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert len(sl) == len(eng.slices(B))
    kern = eng.op_kernels(eng.slices(B)[0], len(rows))
    launching = [i for i, k in enumerate(kern) if k and not k.startswith("(") and "fused into the stem" not in k]
    for t in sl:
        assert sum(t[i] > 0 for i in launching) >= len(launching) // 2, (t, kern)
        assert all(v >= 0 for v in t)
    # grouped launches report on their first op; a slice's launch times tile its stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.profile_insitu(frames, out, cap=len(rows))
    ev[1].record()
    ev[1].synchronize()
    wall = ev[0].elapsed_time(ev[1])
    assert max(sum(t) for t in sl) <= 1.5 * wall + 0.5


def test_insitu_float_input_protonet():
    """the fp32 NCHW entry (the YOLACT protonet line's roofline): 17 frames = two concurrent slices"""
    from tauv_vision_amd.yolact import Masknet, YolactConfig
    m = Masknet(YolactConfig(640, 360, (24, 48, 96, 192, 384), (1,), (0.1, 0.2), feature_depth=64,
                             n_prototype_masks=16), precision="fp16").cuda()
    x = torch.randn(17, 64, 9, 17, generator=torch.Generator().manual_seed(4)).cuda()
    eng = m.engine(torch.device("cuda", 0), 9, 17)
    ref = eng.forward(x)
    rows = eng.profile(x)
    out = torch.empty_like(ref)
    sl = eng.profile_insitu(x, out, cap=len(rows))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert len(sl) == len(eng.slices(17)) and all(sum(t) > 0 for t in sl)
