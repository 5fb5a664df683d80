"""Decode phase stamps (stamp build, lib_d1): shader-clock cycles since the selecting workgroup's
start at each phase boundary, B=1 and B=64 (K=100), from the last records' stamp slots."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tauv-vision_amd")]
from tauv_vision_amd import _lib  # noqa: E402

_lib.set_library_path(os.path.join(ROOT, "tauv-vision_amd", "lib_d1", "libtauv_vision_amd.so"))
import torch  # noqa: E402

from tauv_vision_amd.decode import DeviceDecoder  # noqa: E402

NAMES = ["fill", "nms+compact", "prefilter", "keys stored", "ticket", "keys+minmax", "levels", "candidates",
         "rank", "records"]
g = torch.Generator().manual_seed(1)
for B in (1, 64):
    heat = (torch.randn((B, 4, 120, 160), generator=g) * 3.0).cuda()
    size = torch.randn((B, 120, 160, 2), generator=g).cuda()
    off = torch.rand((B, 120, 160, 2), generator=g).cuda()
    dec = DeviceDecoder(B, 4, 120, 160, 100, torch.device("cuda"))
    rows = []
    for _ in range(5):
        rec, _ = dec(heat, size, off, None, 0, 4, 480, 640, 0.0)
        torch.cuda.synchronize()
        rows.append(rec[:, 98, :].cpu())
    st = torch.stack(rows[1:]).mean(0)  # [B, 10]
    for b in (0, B - 1):
        print(f"B={B} image {b}: " + "  ".join(f"{n} {v:.0f}" for n, v in zip(NAMES, st[b].tolist())))
