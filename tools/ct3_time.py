"""Timing driver for convt3 experiments (run under rocprofv3 --kernel-trace --stats): the protonet's
two ConvTranspose2d layers at B=32 through tv_diag_convt3. argv[1]: library path (optional)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tauv-vision_amd"))
from tauv_vision_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.set_library_path(sys.argv[1])
L = _lib.lib()
tile = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (0, 0)
for (B, C, H, W, N) in [(32, 256, 69, 69, 256), (32, 256, 138, 138, 256)]:
    x = torch.randn(B, H, W, C, device="cuda").half()
    w = torch.randn(C, N, 3, 3) * 0.02
    b = torch.zeros(N)
    out = torch.empty(B, 2 * H, 2 * W, N, device="cuda", dtype=torch.half)
    for _ in range(6):
        _lib.check(L.tv_diag_convt3(ctypes.c_void_p(x.data_ptr()), B, H, W, C, C, ctypes.c_void_p(w.data_ptr()),
                                    ctypes.c_void_p(b.data_ptr()), N, 2, 1, tile[0], tile[1],
                                    ctypes.c_void_p(out.data_ptr()), N, _lib.stream_of(out.device)), "convt3")
torch.cuda.synchronize()
print("ok")
