"""ctypes binding of the in-tree HIP library (include/tauv_vision_amd.h).

The library is the only compute path: if it is missing or no gfx950 device is visible,
calls fail loudly (there is no CPU fallback in this package).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libtauv_vision_amd.so")

TV_OK, TV_EINVAL, TV_ESHAPE, TV_EHIP, TV_ENOTFOUND, TV_ENOMEM = range(6)
DTYPES = {"fp32": 0, "fp16": 1, "bf16": 2, "fp32x3": 3}  # fp32x3: fp32 with each product as three fp16 MFMAs

c_i32, c_i64, c_f32, c_f64, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p


class ModelDesc(ctypes.Structure):
    _fields_ = [("n_levels", c_i32), ("heights", c_i32 * 8), ("channels", c_i32 * 9), ("downsamples", c_i32),
                ("n_heads", c_i32), ("head_channels", c_i32 * 16), ("in_h", c_i32), ("in_w", c_i32),
                ("compute_dtype", c_i32), ("arch", c_i32)]


class WeightView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", c_vp), ("numel", c_i64)]


EXPORTS = {
    "tv_model_param_count": ([ctypes.POINTER(ModelDesc), ctypes.POINTER(c_i32)], c_i32),
    "tv_model_param_info": ([ctypes.POINTER(ModelDesc), c_i32, ctypes.c_char_p, c_i32, ctypes.POINTER(c_i64),
                             ctypes.POINTER(c_i32)], c_i32),
    "tv_model_geometry": ([ctypes.POINTER(ModelDesc), ctypes.POINTER(c_f64), ctypes.POINTER(c_i32),
                           ctypes.POINTER(c_i32), ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)], c_i32),
    "tv_engine_create": ([ctypes.POINTER(ModelDesc), ctypes.POINTER(WeightView), c_i32, c_i32,
                          ctypes.POINTER(c_vp)], c_i32),
    "tv_engine_create_diag": ([ctypes.POINTER(ModelDesc), ctypes.POINTER(WeightView), c_i32, c_i32,
                               ctypes.c_char_p, ctypes.POINTER(c_vp)], c_i32),
    "tv_engine_destroy": ([c_vp], c_i32),
    "tv_engine_prepare": ([c_vp, c_i32, c_vp], c_i32),
    "tv_engine_trim": ([c_vp], c_i32),
    "tv_engine_forward": ([c_vp, c_vp, c_i32, c_vp, c_vp], c_i32),
    "tv_engine_forward_u8": ([c_vp, c_vp, c_i32, c_vp, c_vp], c_i32),
    "tv_engine_profile": ([c_vp, c_vp, c_i32, c_vp, c_vp, ctypes.POINTER(c_f32), ctypes.POINTER(c_f64), c_i32,
                           ctypes.POINTER(c_i32)], c_i32),
    "tv_engine_profile_u8": ([c_vp, c_vp, c_i32, c_vp, c_vp, ctypes.POINTER(c_f32), ctypes.POINTER(c_f64), c_i32,
                              ctypes.POINTER(c_i32)], c_i32),
    "tv_engine_forward_insitu_u8": ([c_vp, c_vp, c_i32, c_vp, c_vp, ctypes.POINTER(c_f32), c_i32,
                                     ctypes.POINTER(c_i32)], c_i32),
    "tv_engine_forward_insitu": ([c_vp, c_vp, c_i32, c_vp, c_vp, ctypes.POINTER(c_f32), c_i32,
                                  ctypes.POINTER(c_i32)], c_i32),
    "tv_engine_set_insitu": ([c_vp, c_i32], c_i32),
    "tv_engine_insitu_read": ([c_vp, c_i32, c_vp, ctypes.POINTER(c_f32), c_i32, ctypes.POINTER(c_i32)], c_i32),
    "tv_engine_op_label": ([c_vp, c_i32], ctypes.c_char_p),
    "tv_engine_op_kernel": ([c_vp, c_i32, c_i32], ctypes.c_char_p),
    "tv_engine_slices": ([c_vp, c_i32, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)], c_i32),
    "tv_preprocess_u8": ([c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp], c_i32),
    "tv_heatmap_nms": ([c_vp, ctypes.POINTER(c_i64), c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp], c_i32),
    "tv_heatmap_topk": ([c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp], c_i32),
    "tv_index_split": ([c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp], c_i32),
    "tv_decode_workspace_size": ([c_i32, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_i64)], c_i32),
    "tv_decode": ([c_vp, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_i64), c_vp,
                   ctypes.POINTER(c_i64), c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp,
                   ctypes.POINTER(c_i64), c_vp, c_vp, c_vp, c_i64, c_vp], c_i32),
    "tv_yolact_box_decode": ([c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_f32, c_vp, c_vp], c_i32),
    "tv_yolact_box_encode": ([c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_f32, c_vp, c_vp], c_i32),
    "tv_yolact_fast_nms": ([c_vp, c_i32, c_i32, c_vp, c_i32, c_f32, c_f32, c_vp, c_vp, c_vp], c_i32),
    "tv_yolact_nms_workspace_size": ([c_i32, c_i32, c_i32, ctypes.POINTER(c_i64)], c_i32),
    "tv_yolact_fast_nms_batched": ([c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_f32, c_f32, c_vp, c_vp, c_vp, c_i64,
                                    c_vp], c_i32),
    "tv_yolact_assemble_mask": ([c_vp, ctypes.POINTER(c_i64), c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp],
                                c_i32),
    "tv_yolact_assemble_masks": ([c_vp, ctypes.POINTER(c_i64), c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32,
                                  c_vp, c_vp], c_i32),
    "tv_yolact_assemble_masks_indexed": ([c_vp, ctypes.POINTER(c_i64), c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32,
                                          c_vp, c_vp, c_i32, c_vp, c_vp], c_i32),
    "tv_train_heatmap": ([c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_f64, c_vp, c_vp], c_i32),
    "tv_train_keypoint_targets": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                                   c_f64, c_f64, c_vp, c_vp, c_vp, c_vp], c_i32),
    "tv_diag_dcn_conv": ([c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32,
                          c_vp, c_vp], c_i32),
    "tv_diag_conv_small": ([c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32,
                            c_vp, c_i32, c_vp], c_i32),
    "tv_diag_convt3": ([c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp,
                        c_i32, c_vp], c_i32),
    "tv_diag_conv1x1": ([c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp], c_i32),
    "tv_diag_conv_burst": ([c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_i32,
                            c_vp], c_i32),
    "tv_diag_burst_plan": ([ctypes.POINTER(c_i32), c_i32, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_i32)], c_i32),
    "tv_last_error": ([], ctypes.c_char_p),
    "tv_version": ([], ctypes.c_char_p),
}

_lib = None
_lock = threading.Lock()


def set_library_path(path):
    """Diagnostics only (kernel A/B experiments): load another build of the library. Must be
    called before the first call into the library; the package reads no environment."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("tauv_vision_amd: the HIP library is already loaded")
    LIB_PATH = path


def lib():
    """Load (once) and return the HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"tauv_vision_amd: HIP library not built ({LIB_PATH}); run "
                                       "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C tauv-vision_amd`")
                handle = ctypes.CDLL(LIB_PATH)
                for name, (args, res) in EXPORTS.items():
                    fn = getattr(handle, name)
                    fn.argtypes = args
                    fn.restype = res
                _lib = handle
    return _lib


def check(rc, what=""):
    if rc == TV_OK:
        return
    msg = lib().tv_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == TV_EINVAL:
        raise ValueError(text)
    if rc == TV_ENOTFOUND:
        raise KeyError(text)
    if rc == TV_ENOMEM:
        raise MemoryError(text)
    raise RuntimeError(text)


def strides(t, n):
    arr = (c_i64 * n)(*[int(s) for s in t.stride()])
    return arr


def stream_of(device):
    import torch
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def require_gpu_tensor(t, name):
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("tauv_vision_amd needs a gfx950 (MI355X) GPU; no HIP device is visible")
    if not t.is_cuda:
        t = t.cuda()
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    return t
