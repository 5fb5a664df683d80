"""DLA-34 B=1 step as bench.latency_b1 runs it (hipGraph replay): argv precision, replays."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

bench.forward_env_knobs(bench.env_knobs())
prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
model, oc, _ = bench.build_model(prec, dev, "dla34")
mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
frames = torch.randint(0, 256, (1, 480, 640, 3), dtype=torch.uint8, device=dev)
r = bench.latency_b1(model, oc, mc, 100, 0.3, dev, frames, n)
print(r, flush=True)
