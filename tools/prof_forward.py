"""Profiling driver: N forwards of the bench workload (R18, 640x480, fp16) for rocprofv3
kernel traces / PMC passes. Usage: python tools/prof_forward.py [--batch 64] [--iters 3] [--model dla34]
(--model yolact: the YOLACT line's step — protonet, box decode, NMS, mask assembly — at B=32)"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import build_model, env_knobs, forward_env_knobs, yolact_setup  # noqa: E402
forward_env_knobs(env_knobs())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--model", default="r18")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.model == "yolact":
        w = yolact_setup(32 if a.batch == 64 else a.batch, a.precision, dev)
        for _ in range(a.iters):
            w["step"]()
        torch.cuda.synchronize()
        print("done", float(w["masks"][0, 0, 0, 0]))  # (no full-tensor reduction in the PMC pass)
        return
    model, oc, sd = build_model(a.precision, dev, a.model)
    frames = torch.randint(0, 256, (a.batch, 480, 640, 3), device=dev, dtype=torch.uint8)
    eng = model.engine(dev, 480, 640)
    out = eng.alloc_out(a.batch)
    for _ in range(a.iters):
        eng.forward_u8(frames, out)
    torch.cuda.synchronize()
    print("done", float(out.float().abs().mean()))


if __name__ == "__main__":
    main()
