"""Per-kernel HIP-event totals of one forward slice (the bench's per-launch roofline pass) for A/B
runs of library builds / diagnostic knobs: python tools/kern_ab.py --tag X [--batch 32] [--model r18]
(TV_LIB=<other build> and TV_* knobs are forwarded explicitly, as bench.py does)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
bench.forward_env_knobs(bench.env_knobs())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--model", default="r18")
    ap.add_argument("--tag", default="")
    ap.add_argument("--ops", default="", help="also write the per-op best times (JSON) here")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, oc, sd = bench.build_model(a.precision, dev, a.model)
    g = torch.Generator(device=dev).manual_seed(1000)
    frames = torch.randint(0, 256, (a.batch, 480, 640, 3), generator=g, device=dev, dtype=torch.uint8)
    eng = model.engine(dev, 480, 640)
    out = eng.alloc_out(a.batch)
    best = None
    for _ in range(a.reps):
        ops = eng.profile(frames, out)
        best = [list(o) for o in ops] if best is None else [[b[0], min(b[1], o[1]), b[2], b[3]] for b, o in zip(best, ops)]
    kern = {}
    for lab, ms, fl, k in best:
        e = kern.setdefault(k, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += ms
        e[2] += fl
    res = {"tag": a.tag, "model": a.model, "batch": a.batch, "total_ms": round(sum(o[1] for o in best), 4),
           "kernels": {k: {"n": v[0], "ms": round(v[1], 4), "tflops": round(v[2] / max(v[1], 1e-9) / 1e9, 1)}
                       for k, v in sorted(kern.items(), key=lambda kv: -kv[1][1])}}
    print(json.dumps(res), flush=True)
    if a.ops:
        with open(a.ops, "w") as f:
            json.dump([{"op": o[0], "ms": o[1], "gflop": o[2] / 1e9, "kernel": o[3]} for o in best], f, indent=0)


if __name__ == "__main__":
    main()
