"""Per-op HIP-event times of the bench workload (B=64 u8 frames, R18 640x480) for A/B runs of
engine knobs (TV_STEM, TV_CONVT, ... — the names engine.cpp accepts): prints the ops whose label matches --match.
Usage: python tools/op_bench.py [--match projection_layer] [--reps 5] [--precision fp16]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import build_model, env_knobs, forward_env_knobs  # noqa: E402
forward_env_knobs(env_knobs())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--match", default="")
    ap.add_argument("--tag", default="")
    ap.add_argument("--dump", default="", help="write the op labels as JSON (tools/stamps.py)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, oc, sd = build_model(a.precision, dev)
    frames = torch.randint(0, 256, (a.batch, 480, 640, 3), device=dev, dtype=torch.uint8)
    eng = model.engine(dev, 480, 640)
    out = eng.alloc_out(a.batch)
    best = None
    for _ in range(a.reps):
        ops = eng.profile(frames, out)
        best = [list(o) for o in ops] if best is None else [[b[0], min(b[1], o[1]), b[2], b[3]] for b, o in zip(best, ops)]
    tot = sum(o[1] for o in best)
    if a.dump:
        import json
        with open(a.dump, "w") as f:
            json.dump([{"op": o[0]} for o in best], f)
    sel = [o for o in best if a.match in o[0]]
    for o in sel:
        print(f"{a.tag} {o[1]:8.4f} ms {o[2] / max(o[1], 1e-9) / 1e9:8.1f} TF  {o[3][:40]:40s} {o[0][:60]}")
    print(f"{a.tag} total {tot:.3f} ms")


if __name__ == "__main__":
    main()
