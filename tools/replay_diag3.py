"""Diagnostic: B=1 graph replays vs eager under kernel-choice knobs (which kernel breaks replays)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tauv_vision_amd import engine as E  # noqa: E402

VARIANTS = [{}, {"TV_LAT": "0"}, {"TV_CONVT": "0"}, {"TV_STEMFUSE": "0"}, {"TV_HEADFUSE": "0"}, {"TV_C1X1": "0"},
            {"TV_C3_NW": "8"}, {"TV_CONV3": "0", "TV_CONV3S2": "0"},
            {"TV_LAT": "0", "TV_CONVT": "0", "TV_STEMFUSE": "0", "TV_HEADFUSE": "0", "TV_C1X1": "0"}]


def one(knobs, arch="r18", precision="fp16", n=6):
    E._DIAG_KNOBS = dict(knobs)
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model(precision, dev, arch)
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
    frame = torch.randint(0, 256, (1, 480, 640, 3), generator=torch.Generator().manual_seed(105),
                          dtype=torch.uint8).to(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        out = torch.empty_like(model.engine(dev, 480, 640).alloc_out(1))
        eng = model.engine(dev, 480, 640)
        eng.prepare(1)
        for _ in range(2):
            eng.forward_u8(frame, out)
        s.synchronize()
        ref = out.clone()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        eng.forward_u8(frame, out)
    bad = []
    for _ in range(n):
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        bad.append(int(not torch.equal(out, ref)))
    kinds = sorted({k.split("<")[0] for _, _, _, k in eng.profile(frame, eng.alloc_out(1))})
    print(json.dumps({"knobs": knobs, "bad": bad, "kernels": kinds}), flush=True)
    del g, eng, model
    torch.cuda.synchronize()


if __name__ == "__main__":
    for v in VARIANTS:
        one(v)
