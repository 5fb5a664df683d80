"""Diagnostic: where conv_burst leaves outputs unwritten / wrong (single 3x3 layer via the diag entry)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
from test_gpu_conv_burst import _diag_burst, _ref  # noqa: E402

B, Ho, Wo, N = 2, 15, 20, 128
g = torch.Generator().manual_seed(1)
x = torch.randn(B, 128, Ho, Wo, generator=g).half().float()
w = (torch.randn(N, 1152, generator=g) / 34).half().float()
b = torch.randn(N, generator=g) * 0.1
got = _diag_burst([(x, 3, 1)], B, Ho, Wo, w, b, 0, "fp16")
ref = _ref([(x, 3, 1)], w, b, 0)
nan = torch.isnan(got)
print("nan count", int(nan.sum()), "of", nan.numel())
print("nan per channel (first 40):", nan.sum(dim=(0, 2, 3))[:40].tolist())
print("nan per frame:", nan.sum(dim=(1, 2, 3)).tolist())
pix = nan.any(dim=1)  # [B, Ho, Wo]
print("nan pixels frame0 rows:", pix[0].sum(dim=1).tolist())
err = (got - ref).abs().nan_to_num(-1)
ok = (err >= 0) & (err < 1e-2)
print("ok fraction", float(ok.float().mean()))
print("bad (non-nan) per row frame0:", ((err >= 1e-2).any(dim=1))[0].sum(dim=1).tolist())
print("sample got/ref [0,0,5,5]", got[0, :4, 5, 5].tolist(), ref[0, :4, 5, 5].tolist())
