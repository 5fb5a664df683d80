"""Per-launch HIP-event times of one R18 forward at batch 1 (the latency path), grouped by kernel."""
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tauv-vision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
bench.forward_env_knobs(bench.env_knobs())
import tauv_vision_amd as tv  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
arch = os.environ.get("OPS_MODEL", "r18")
dev = torch.device("cuda", 0)
model, oc, _ = bench.build_model(prec, dev, arch)
eng = model.engine(dev, 480, 640)
fr = torch.randint(0, 256, (B, 480, 640, 3), dtype=torch.uint8, device=dev)
out = eng.alloc_out(B)
best = None
for _ in range(5):
    ops = eng.profile(fr, out)
    if best is None:
        best = [list(o) for o in ops]
    else:
        for b, o in zip(best, ops):
            b[1] = min(b[1], o[1])
tot = sum(o[1] for o in best)
print(f"B={B} {prec}: {len(best)} launches, {tot:.3f} ms summed")
k = defaultdict(lambda: [0, 0.0])
for o in best:
    k[o[3]][0] += 1
    k[o[3]][1] += o[1]
for n, v in sorted(k.items(), key=lambda kv: -kv[1][1]):
    print(f"{v[1]:7.3f} ms {v[0]:3d} x {1e3 * v[1] / v[0]:6.1f} us  {n}")
if len(sys.argv) > 3:
    json.dump([{"op": o[0], "ms": o[1], "gflop": o[2] / 1e9, "kernel": o[3]} for o in best], open(sys.argv[3], "w"), indent=0)
