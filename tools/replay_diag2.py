"""Diagnostic: which part of the B=1 captured step goes wrong on replays after the first."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def setup(arch="r18", precision="fp16"):
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model(precision, dev, arch)
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
    frame = torch.randint(0, 256, (1, 480, 640, 3), generator=torch.Generator().manual_seed(105),
                          dtype=torch.uint8).to(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        pipe = bench.Pipeline(model, oc, mc, 1, 100, 0.0, dev)
        for _ in range(2):
            pipe.step(frame)
        s.synchronize()
        ref = pipe.out.clone()
    torch.cuda.current_stream(dev).wait_stream(s)
    return pipe, frame, s, ref


def replays(pipe, ref, g, fill, n=8, sync_each=True):
    bad = []
    for _ in range(n):
        if fill:
            pipe.out.fill_(float("nan"))
        g.replay()
        if sync_each:
            torch.cuda.synchronize()
        bad.append(int(not torch.equal(pipe.out, ref)))
    torch.cuda.synchronize()
    return bad


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    pipe, frame, s, ref = setup()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pipe.step(frame)
    print(json.dumps({"tag": tag, "variant": "step, nan fill", "bad": replays(pipe, ref, g, True)}), flush=True)
    print(json.dumps({"tag": tag, "variant": "step, no fill", "bad": replays(pipe, ref, g, False)}), flush=True)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s):
        pipe.eng.forward_u8(frame, pipe.out)
    print(json.dumps({"tag": tag, "variant": "forward only, nan fill", "bad": replays(pipe, ref, g2, True)}), flush=True)
    # eager after the graphs: still right?
    with torch.cuda.stream(s):
        pipe.out.fill_(float("nan"))
        pipe.eng.forward_u8(frame, pipe.out)
        s.synchronize()
    print(json.dumps({"tag": tag, "variant": "eager after", "bad": [int(not torch.equal(pipe.out, ref))]}), flush=True)


if __name__ == "__main__":
    main()
