import os, sys
ROOT = os.environ["GRAFT_REPO_ROOT"]
sys.path[:0] = [ROOT, os.path.join(ROOT, "tauv-vision_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch
from helpers import golden, dla34_input
from test_gpu_dla34 import build
name = "b1_480x640_kp"
model, oc, mc, case = build(name, "fp16")
with torch.no_grad():
    pred = model(dla34_input(name).cuda())
g = golden(f"dla34_{name}")
err = np.abs(pred.heatmap.float().cpu().numpy() - g["heatmap"])[0]   # [C, H, W]
print("max", err.max(), "mean", err.mean())
c, y, x = np.unravel_index(np.argsort(err.ravel())[-20:], err.shape)
print(list(zip(c, y, x)))
e2 = err.max(0)
print("rows max", [round(float(v), 6) for v in e2.max(1)[::8]])
print("cols max", [round(float(v), 6) for v in e2.max(0)[::8]])
big = e2 > 3e-4
print("frac big", big.mean(), "rows", np.nonzero(big.any(1))[0][:40], "cols", np.nonzero(big.any(0))[0][:40])
