"""dcn_win phase stamps (stamp build: make BUILD=build_s LIBDIR=lib_s EXTRA=-DTV_DCN_STAMPS=1): per-wave
shader-clock cycles per bucket over one 120x160 64 -> 64 DeformConv at B=32 (DLA-34's node layers),
offsets of sigma 0.5 (the trained-like field), averaged over the workgroups' waves."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tauv-vision_amd")]
from tauv_vision_amd import _lib  # noqa: E402

_lib.set_library_path(os.path.join(ROOT, "tauv-vision_amd", "lib_s", "libtauv_vision_amd.so"))
import torch  # noqa: E402

NAMES = ["tile-top wait", "sampling state", "corners+blend", "MFMAs", "tap-8 barrier+issue", "epilogue", "tiles"]
B, C, H, W, N = 32, 64, 120, 160, 64
g = torch.Generator().manual_seed(3)
x = torch.randn(B, H, W, C, generator=g).half().cuda()
om = torch.zeros(B, H, W, 32)
om[..., :18] = torch.randn(B, H, W, 18, generator=g) * 0.5
om[..., 18:27] = torch.randn(B, H, W, 9, generator=g)
om = om.half().cuda()
w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).contiguous()
b = torch.zeros(N)
out = torch.empty(B, H, W, N, dtype=torch.float16, device="cuda")
L = _lib.lib()
for rep in range(3):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    _lib.check(L.tv_diag_dcn_conv(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(om.data_ptr()), B, H, W, C, 32,
                                  ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(b.data_ptr()), N, 1, 1, 4,
                                  ctypes.c_void_p(out.data_ptr()), _lib.stream_of(out.device)), "dcn")
    ev[1].record()
    torch.cuda.synchronize()
    print(f"call {rep}: {ev[0].elapsed_time(ev[1]) * 1e3:.1f} us (diag: includes weight upload)")
st = out.view(torch.int64).view(-1)[:256 * 8 * 8].view(256, 8, 8).cpu().double()
m = st.mean((0, 1))
tot = float(m[:6].sum())
print("per wave, mean over 256 workgroups x 8 waves: total %.0f cycles, %.1f tiles" % (tot, float(m[6])))
for i in range(6):
    print(f"  {NAMES[i]:22s} {float(m[i]):10.0f} cycles  {100 * float(m[i]) / tot:5.1f}%  ({float(m[i]) / max(1, float(m[6])):8.0f} per tile)")
