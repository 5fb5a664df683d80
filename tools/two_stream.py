"""Experiment: the B=64 step split into S concurrent streams of B/S frames each (forward_u8 only).
Usage: python tools/two_stream.py [--splits 1 2 4] [--steps 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import build_model, env_knobs, forward_env_knobs  # noqa: E402
forward_env_knobs(env_knobs())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, oc, sd = build_model("fp16", dev)
    frames = torch.randint(0, 256, (a.batch, 480, 640, 3), device=dev, dtype=torch.uint8)
    eng = model.engine(dev, 480, 640)
    for S in a.splits:
        b = a.batch // S
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        outs = [eng.alloc_out(b) for _ in range(S)]
        parts = [frames[i * b:(i + 1) * b] for i in range(S)]

        def step():
            cur = torch.cuda.current_stream(dev)
            for i in range(S):
                streams[i].wait_stream(cur)
                with torch.cuda.stream(streams[i]):
                    eng.forward_u8(parts[i], outs[i])
            for i in range(S):
                cur.wait_stream(streams[i])
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"splits {S}: {el / a.steps * 1e3:.3f} ms/step, {a.batch * a.steps / el:.1f} fps", flush=True)


if __name__ == "__main__":
    main()
