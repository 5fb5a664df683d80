"""Decode timing probe: DeviceDecoder (peak_scan + peak_select) on a real R18 head tensor
and on random logits, B in {1, 64}, K in {1, 10, 100}; HIP-event time per call (min of 20)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tauv-vision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import tauv_vision_amd as tv  # noqa: E402
from tauv_vision_amd.decode import DeviceDecoder  # noqa: E402


def t_call(fn, reps=20):
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    best = 1e9
    for _ in range(reps):
        ev[0].record(s)
        fn()
        ev[1].record(s)
        ev[1].synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]))
    return best * 1e3


dev = torch.device("cuda", 0)
model, oc, _ = bench.build_model("fp16", dev)
mc = tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, 2, 1.0)
frames = torch.randint(0, 256, (64, 480, 640, 3), dtype=torch.uint8, device=dev)
pipe = bench.Pipeline(model, oc, mc, 64, 100, 0.3, dev)
pipe.eng.forward_u8(frames, pipe.out)
p = pipe.pred
only = "--only" in sys.argv  # the bench configuration alone (B=64, K=100, R18 heads)
only1 = "--only1" in sys.argv  # the B=1 latency configuration alone
for name, heat in (("r18", p.heatmap), ("rand", (torch.rand_like(p.heatmap) * 9 - 8)))[:1 if only or only1 else 2]:
    for B in ((64,) if only else (1,) if only1 else (64, 1)):
        for K in ((100,) if only or only1 else (100, 10, 1)):
            d = DeviceDecoder(B, 4, 120, 160, K, dev)
            us = t_call(lambda: d(heat[:B], p.size[:B], p.offset[:B], None, 0, 4, 480, 640, 0.3))
            print(f"{name:5s} B={B:3d} K={K:3d}: {us:8.1f} us", flush=True)
