"""Owning wrapper of one native engine (tv_engine_*): built from reference-layout weights
for one (device, input size, precision); forward launches on the caller's torch stream."""
import ctypes

import torch

from . import _lib
from .weights import geometry


_DIAG_KNOBS = {}


def set_diagnostic_knobs(knobs):
    """Diagnostics only (kernel A/B experiments): kernel-choice overrides ({"TV_C3_TW": "16", ...},
    the names engine.cpp lists) for engines created after this call, through
    tv_engine_create_diag. The product path passes none and reads no environment."""
    global _DIAG_KNOBS
    _DIAG_KNOBS = {str(k): str(v) for k, v in (knobs or {}).items()}


class NativeEngine:
    def __init__(self, desc, state_dict, device_index):
        self.desc = desc
        self.device = torch.device("cuda", device_index)
        self.geom = geometry(desc)
        host = {k: v.detach().to("cpu", torch.float32).contiguous() for k, v in state_dict.items()
                if v.dtype.is_floating_point}
        views = (_lib.WeightView * len(host))()
        keep = []
        for i, (k, v) in enumerate(host.items()):
            name = k.encode()
            keep.append(name)
            views[i].name = name
            views[i].data = v.data_ptr()
            views[i].numel = v.numel()
        handle = ctypes.c_void_p()
        L = _lib.lib()
        with torch.cuda.device(self.device):
            if _DIAG_KNOBS:
                spec = ";".join(f"{k}={v}" for k, v in sorted(_DIAG_KNOBS.items())).encode()
                rc = L.tv_engine_create_diag(ctypes.byref(desc), views, len(host), device_index, spec,
                                             ctypes.byref(handle))
            else:
                rc = L.tv_engine_create(ctypes.byref(desc), views, len(host), device_index, ctypes.byref(handle))
            _lib.check(rc, "engine create")
        self._h = handle
        self.generation = 0  # bumped by trim(): graphs captured before it reference freed workspaces
        del keep, host

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.tv_engine_destroy(h)
            self._h = None

    @property
    def out_shape_per_frame(self):
        g = self.geom
        return g["out_h"], g["out_w"], g["out_cpad"]

    def slices(self, batch):
        """Frame counts of the concurrent slices a forward of `batch` frames launches."""
        n = ctypes.c_int32()
        sb = (ctypes.c_int32 * 8)()  # TV_MAX_SLICES
        _lib.check(_lib.lib().tv_engine_slices(self._h, batch, ctypes.byref(n), sb), "slices")
        return [sb[i] for i in range(n.value)]

    def op_kernels(self, batch, n):
        """Kernel instance of each of the first n ops in a `batch`-frame workspace ("" before it exists)."""
        L = _lib.lib()
        return [L.tv_engine_op_kernel(self._h, batch, i).decode() for i in range(n)]

    def alloc_out(self, batch):
        oh, ow, oc = self.out_shape_per_frame
        return torch.empty((batch, oh, ow, oc), dtype=torch.float32, device=self.device)

    def prepare(self, batch):
        _lib.check(_lib.lib().tv_engine_prepare(self._h, int(batch), _lib.stream_of(self.device)), "prepare")

    def trim(self):
        """Free every cached (stream, batch) workspace (synchronises the device)."""
        _lib.check(_lib.lib().tv_engine_trim(self._h), "trim")
        self.generation += 1

    def forward(self, img, out=None):
        """img: fp32 NCHW on this device; returns the fp32 NHWC head tensor."""
        B = img.shape[0]
        if out is None:
            out = self.alloc_out(B)
        if B == 0:  # an empty batch: nothing to launch (the reference's convolutions return empty outputs)
            return out
        _lib.check(_lib.lib().tv_engine_forward(self._h, ctypes.c_void_p(img.data_ptr()), B,
                                                ctypes.c_void_p(out.data_ptr()), _lib.stream_of(self.device)),
                   "forward")
        return out

    def forward_u8(self, frames, out=None):
        """frames: uint8 NHWC RGB on this device (ToTensor + ImageNet Normalize fused)."""
        B = frames.shape[0]
        if out is None:
            out = self.alloc_out(B)
        if B == 0:
            return out
        _lib.check(_lib.lib().tv_engine_forward_u8(self._h, ctypes.c_void_p(frames.data_ptr()), B,
                                                   ctypes.c_void_p(out.data_ptr()), _lib.stream_of(self.device)),
                   "forward_u8")
        return out

    def profile_insitu(self, frames, out=None, cap=1024):
        """One forward as it runs (concurrent slices, grouped launches), an event before each launch
        on its slice's stream: per slice, per op index the launch's ms (0 for ops that launch nothing
        of their own). `frames`: uint8 NHWC (forward_u8) or the fp32 NCHW forward() input."""
        B = frames.shape[0]
        if out is None:
            out = self.alloc_out(B)
        ns = ctypes.c_int32()
        ms = (ctypes.c_float * (cap * 8))()
        L = _lib.lib()
        fn = L.tv_engine_forward_insitu_u8 if frames.dtype == torch.uint8 else L.tv_engine_forward_insitu
        _lib.check(fn(self._h, ctypes.c_void_p(frames.data_ptr()), B, ctypes.c_void_p(out.data_ptr()),
                      _lib.stream_of(self.device), ms, cap, ctypes.byref(ns)), "forward_insitu")
        return [[ms[k * cap + i] for i in range(cap)] for k in range(ns.value)]

    def set_insitu(self, on):
        """Record the per-launch group events in every forward (also into a graph captured meanwhile)."""
        _lib.check(_lib.lib().tv_engine_set_insitu(self._h, 1 if on else 0), "set_insitu")

    def insitu_read(self, batch, stream, cap=1024):
        """Per slice, per op index: the launch times the `batch`-frame forward keyed to `stream` (a
        torch stream; a graph's capture stream) last recorded."""
        ns = ctypes.c_int32()
        ms = (ctypes.c_float * (cap * 8))()
        _lib.check(_lib.lib().tv_engine_insitu_read(self._h, batch, ctypes.c_void_p(stream.cuda_stream), ms, cap,
                                                    ctypes.byref(ns)), "insitu_read")
        return [[ms[k * cap + i] for i in range(cap)] for k in range(ns.value)]

    def profile(self, img, out=None, cap=4096):
        """Per-launch (label, ms, flops, kernel) of one forward, timed with HIP events. `img` is the
        normalised fp32 NCHW input of forward() or uint8 NHWC frames (the forward_u8 path)."""
        B = img.shape[0]
        if out is None:
            out = self.alloc_out(B)
        ms = (ctypes.c_float * cap)()
        fl = (ctypes.c_double * cap)()
        n = ctypes.c_int32()
        L = _lib.lib()
        fn = L.tv_engine_profile_u8 if img.dtype == torch.uint8 else L.tv_engine_profile
        _lib.check(fn(self._h, ctypes.c_void_p(img.data_ptr()), B, ctypes.c_void_p(out.data_ptr()),
                                       _lib.stream_of(self.device), ms, fl, cap, ctypes.byref(n)), "profile")
        return [(L.tv_engine_op_label(self._h, i).decode(), ms[i], fl[i], L.tv_engine_op_kernel(self._h, B, i).decode())
                for i in range(min(n.value, cap))]
