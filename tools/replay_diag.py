"""Diagnostic: determinism of the B=1 step, eager and as a replayed hipGraph, under engine knobs
(TV_LAT_SPLIT=1: no conv_lat split-K; TV_LATGROUP=0: plan order). Prints mismatch counts."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tauv_vision_amd import engine as E  # noqa: E402


def run(knobs, arch="r18", precision="fp16", n=12):
    E._DIAG_KNOBS = dict(knobs)
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model(precision, dev, arch)
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
    frame = torch.randint(0, 256, (1, 480, 640, 3), generator=torch.Generator().manual_seed(105),
                          dtype=torch.uint8).to(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    res = {"knobs": knobs}
    with torch.cuda.stream(s):
        pipe = bench.Pipeline(model, oc, mc, 1, 100, 0.0, dev)
        pipe.step(frame)
        s.synchronize()
        ref = pipe.out.clone()
        bad = 0
        for _ in range(n):
            pipe.out.fill_(float("nan"))
            pipe.step(frame)
            s.synchronize()
            bad += int(not torch.equal(pipe.out, ref))
        res["eager_mismatch"] = bad
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pipe.step(frame)
    bad, maxd = 0, 0.0
    for _ in range(n):
        pipe.out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        if not torch.equal(pipe.out, ref):
            bad += 1
            maxd = max(maxd, float((pipe.out - ref).abs().nan_to_num(1e9).max()))
    res["replay_mismatch"] = bad
    res["replay_maxdiff"] = maxd
    # ops whose kernel runs split-K / grouped: names
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    for kn in ({}, {"TV_LAT_SPLIT": "1"}, {"TV_LATGROUP": "0"}, {"TV_LAT_SPLIT": "1", "TV_LATGROUP": "0"}):
        run(kn)
