"""Drop-in YOLACT protonet and post-processing (reference
src/tauv_vision/yolact/model/): `Masknet` (masknet.py:8-55), `get_anchor` (anchors.py:9-41),
`box_encode` / `box_decode` (boxes.py:45-61), `nms` (nms.py:7-29) and `assemble_mask`
(masks.py:8-21), as called by the YOLACT node (yolact_node.py:118-134), plus batched forms of
nms / assemble_mask for B images at once.

Masknet, box_encode/decode, nms and assemble_mask run in the HIP library (csrc/) on the tensors'
GPU; there is no CPU fallback. `get_anchor` builds the per-level anchor constants on the host
exactly like the reference (it is configuration, computed once per FPN level).
"""
from dataclasses import dataclass
from math import sqrt
from typing import Optional, Tuple

import ctypes
import torch
import torch.nn as nn

from . import _lib
from .dla import populate
from .engine import NativeEngine
from .weights import param_layout, protonet_desc


@dataclass
class YolactConfig:
    """The fields of the reference yolact ModelConfig (config.py:8-40) the protonet and the
    post-processing read."""
    in_w: int
    in_h: int
    anchor_scales: Tuple[int, ...]
    anchor_aspect_ratios: Tuple[float, ...]
    box_variances: Tuple[float, float]
    feature_depth: int = 256
    n_prototype_masks: int = 8


class Masknet(nn.Module):
    """masknet.py:8-55: fpn[0] [B, F, H, W] -> prototypes [B, k, 4H, 4W] (LeakyReLU output).

    Parameters keep the reference key layout (`_layers_1.0.0.weight`, `_upsample_layer_1.weight`,
    ..., `_output_layer.bias`), so `load_state_dict` of a reference Masknet (or of the `_masknet.`
    sub-dict of a Yolact checkpoint) works unchanged. The forward pass is one native call: the
    3x3 convs as MFMA implicit GEMMs, each ConvTranspose2d(3, s2, p1) as four phase GEMMs (one per
    output parity, exactly its 9 taps per 2x2 block), bias + LeakyReLU in the epilogues. The result
    is a [B, k, 4H, 4W] view of one fp32 NHWC tensor (the layout assemble_mask reads fastest).
    `precision`: "fp32" (exact-f32 MFMA, parity mode), "fp16" or "bf16" (fp32 accumulation)."""

    def __init__(self, config, precision: str = "fp32"):
        super().__init__()
        self.feature_depth = int(config.feature_depth)
        self.n_prototype_masks = int(config.n_prototype_masks)
        if precision not in _lib.DTYPES:
            raise ValueError(f"precision must be one of {sorted(_lib.DTYPES)}")
        self.precision = precision
        layout = param_layout(protonet_desc(self.feature_depth, self.n_prototype_masks))
        populate(self, layout, seed_layout=layout)
        self._version = 0
        self._engines = {}
        self.register_load_state_dict_post_hook(lambda module, keys: module.invalidate())

    def invalidate(self):
        self._version += 1
        self._engines = {}

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self.invalidate()
        return r

    def engine(self, device: torch.device, fpn_h: int, fpn_w: int) -> NativeEngine:
        key = (device.index if device.index is not None else torch.cuda.current_device(), fpn_h, fpn_w,
               self.precision, self._version)
        eng = self._engines.get(key)
        if eng is None:
            desc = protonet_desc(self.feature_depth, self.n_prototype_masks, fpn_h, fpn_w, self.precision)
            eng = NativeEngine(desc, self.state_dict(), key[0])
            self._engines = {key: eng}
        return eng

    def forward_nhwc(self, fpn_output: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The native result: fp32 NHWC [B, 4H, 4W, k rounded up to 4]."""
        if fpn_output.dim() != 4 or fpn_output.shape[1] != self.feature_depth:
            raise ValueError(f"expected fpn_output [batch, {self.feature_depth}, H, W], got {tuple(fpn_output.shape)}")
        if not torch.cuda.is_available():
            raise RuntimeError("tauv_vision_amd needs a gfx950 (MI355X) GPU; no HIP device is visible")
        dev = fpn_output.device if fpn_output.is_cuda else torch.device("cuda", torch.cuda.current_device())
        x = fpn_output.to(dev, torch.float32).contiguous()
        return self.engine(dev, x.shape[2], x.shape[3]).forward(x, out)

    def forward(self, fpn_output: torch.Tensor) -> torch.Tensor:
        return self.forward_nhwc(fpn_output)[..., :self.n_prototype_masks].permute(0, 3, 1, 2)


def get_anchor(fpn_i: int, fpn_size, config) -> torch.Tensor:
    """anchors.py:9-41: [1, H*W*n_ar, 4] (y, x, h, w) at cell centres; per aspect ratio a block."""
    n = len(config.anchor_aspect_ratios)
    y = (torch.arange(0, fpn_size[0]) + 0.5) / fpn_size[0]
    x = (torch.arange(0, fpn_size[1]) + 0.5) / fpn_size[1]
    y, x = torch.meshgrid(y, x, indexing="ij")
    y = torch.tile(y.flatten(), (1, n))
    x = torch.tile(x.flatten(), (1, n))
    scale = config.anchor_scales[fpn_i]
    in_size = (config.in_h + config.in_w) / 2
    hw = fpn_size[0] * fpn_size[1]
    h = torch.cat([torch.full((1, hw), (scale / in_size) * sqrt(ar)) for ar in config.anchor_aspect_ratios], -1)
    w = torch.cat([torch.full((1, hw), (scale / in_size) / sqrt(ar)) for ar in config.anchor_aspect_ratios], -1)
    return torch.stack((y, x, h, w), dim=1).permute(0, 2, 1)


def _f32(t, name):
    return _lib.require_gpu_tensor(t, name).contiguous()


def _boxes_op(fn, name, a: torch.Tensor, anchor: torch.Tensor, config) -> torch.Tensor:
    x = _f32(a, name)
    anc = _f32(anchor, "anchor").to(x.device)
    if x.dim() != 3 or x.shape[-1] != 4 or anc.dim() != 3 or anc.shape[1:] != x.shape[1:]:
        raise ValueError(f"{name}: {tuple(x.shape)} / anchors {tuple(anc.shape)} mismatch")
    out = torch.empty_like(x)
    B, A, _ = x.shape
    _lib.check(fn(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(anc.data_ptr()), B, A, anc.shape[0],
                  float(config.box_variances[0]), float(config.box_variances[1]), ctypes.c_void_p(out.data_ptr()),
                  _lib.stream_of(x.device)), name)
    return out


def box_decode(box_encoding: torch.Tensor, anchor: torch.Tensor, config) -> torch.Tensor:
    """boxes.py:55-61 on the GPU: [B, A, 4] encodings + [1 or B, A, 4] anchors -> boxes (y, x, h, w)."""
    return _boxes_op(_lib.lib().tv_yolact_box_decode, "box_decode", box_encoding, anchor, config)


def box_encode(box: torch.Tensor, anchor: torch.Tensor, config) -> torch.Tensor:
    """boxes.py:45-53 on the GPU: [B, A, 4] boxes (y, x, h, w) + [1 or B, A, 4] anchors -> encodings."""
    return _boxes_op(_lib.lib().tv_yolact_box_encode, "box_encode", box, anchor, config)


def _nms_args(classification, box):
    cls = _f32(classification, "classification")
    bx = _f32(box, "box").to(cls.device)
    if cls.dim() != 3 or bx.dim() != 3 or bx.shape[-1] != 4 or cls.shape[1] != bx.shape[1]:
        raise ValueError(f"nms: classification {tuple(cls.shape)} / box {tuple(bx.shape)} mismatch")
    return cls, bx


def nms(classification: torch.Tensor, box: torch.Tensor, top_k: int, iou_threshold: float,
        confidence_threshold: float) -> torch.Tensor:
    """nms.py:7-29 (YOLACT fast NMS, batch 0 only): int64 indices of the kept anchors in
    descending-confidence order. Any anchor count. One device->host read of the kept count."""
    cls, bx = _nms_args(classification, box)
    A, C1 = cls.shape[1], cls.shape[2]
    K = min(int(top_k), A)
    det = torch.empty((max(K, 1),), dtype=torch.int64, device=cls.device)
    n = torch.empty((1,), dtype=torch.int32, device=cls.device)
    _lib.check(_lib.lib().tv_yolact_fast_nms(ctypes.c_void_p(cls[0].data_ptr()), A, C1, ctypes.c_void_p(bx[0].data_ptr()),
                                             int(top_k), float(iou_threshold), float(confidence_threshold),
                                             ctypes.c_void_p(det.data_ptr()), ctypes.c_void_p(n.data_ptr()),
                                             _lib.stream_of(cls.device)), "nms")
    return det[:int(n.item())]


class BatchedNMS:
    """nms.py:7-29 applied to every image of a [B, A, C+1] / [B, A, 4] batch with static device
    buffers (graph-capturable, no host sync): returns (det [B, min(top_k, A)] int64 — row b's first
    counts[b] entries are its kept anchors in descending confidence —, counts [B] int32)."""

    def __init__(self, B, A, top_k, device):
        self.B, self.A, self.top_k = int(B), int(A), int(top_k)
        self.K = min(self.top_k, self.A)
        nbytes = ctypes.c_int64()
        _lib.check(_lib.lib().tv_yolact_nms_workspace_size(self.B, self.A, self.top_k, ctypes.byref(nbytes)),
                   "nms workspace")
        self.ws = torch.empty((max(nbytes.value, 256),), dtype=torch.uint8, device=device)
        self.det = torch.zeros((self.B, self.K), dtype=torch.int64, device=device)
        self.counts = torch.zeros((self.B,), dtype=torch.int32, device=device)

    def __call__(self, classification, box, iou_threshold, confidence_threshold):
        cls, bx = _nms_args(classification, box)
        if cls.shape[0] != self.B or cls.shape[1] != self.A:
            raise ValueError(f"BatchedNMS built for [{self.B}, {self.A}], got {tuple(cls.shape)}")
        _lib.check(_lib.lib().tv_yolact_fast_nms_batched(
            ctypes.c_void_p(cls.data_ptr()), self.B, self.A, cls.shape[2], ctypes.c_void_p(bx.data_ptr()), self.top_k,
            float(iou_threshold), float(confidence_threshold), ctypes.c_void_p(self.det.data_ptr()),
            ctypes.c_void_p(self.counts.data_ptr()), ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(),
            _lib.stream_of(cls.device)), "nms_batched")
        return self.det, self.counts


def _proto_view(t, name):
    t = _lib.require_gpu_tensor(t, name)
    if t.stride()[-1] != 1 and t.stride()[-3] != 1:
        t = t.contiguous()
    return t


def assemble_mask(mask_prototype: torch.Tensor, mask_coeff: torch.Tensor,
                  box: Optional[torch.Tensor]) -> torch.Tensor:
    """masks.py:8-21: prototypes [K, H, W] (any strides: NCHW slices or Masknet's NHWC view),
    coefficients [n, K], boxes [n, 4] or None -> [n, H, W]."""
    proto = _proto_view(mask_prototype, "mask_prototype")
    coeff = _f32(mask_coeff, "mask_coeff").to(proto.device)
    if proto.dim() != 3 or coeff.dim() != 2 or coeff.shape[1] != proto.shape[0]:
        raise ValueError(f"assemble_mask: prototypes {tuple(proto.shape)} / coefficients {tuple(coeff.shape)} mismatch")
    bptr = None
    if box is not None:
        box = _f32(box, "box").to(proto.device)
        if box.shape != (coeff.shape[0], 4):
            raise ValueError(f"assemble_mask: box {tuple(box.shape)} must be [n, 4]")
        bptr = ctypes.c_void_p(box.data_ptr())
    K, H, W = proto.shape
    n = coeff.shape[0]
    out = torch.empty((n, H, W), dtype=torch.float32, device=proto.device)
    if n == 0:  # no detections (the node returns before this, yolact_node.py:131-133)
        return out
    _lib.check(_lib.lib().tv_yolact_assemble_mask(ctypes.c_void_p(proto.data_ptr()), _lib.strides(proto, 3), K, H, W,
                                                  ctypes.c_void_p(coeff.data_ptr()), bptr, n,
                                                  ctypes.c_void_p(out.data_ptr()), _lib.stream_of(proto.device)),
               "assemble_mask")
    return out


def _check_out(out, shape, device, what):
    """A caller-supplied output: the kernel writes [B, n, H, W] fp32 through its raw pointer."""
    if out is None:
        return torch.empty(shape, dtype=torch.float32, device=device)
    if tuple(out.shape) != tuple(shape) or out.dtype != torch.float32 or not out.is_contiguous() \
            or out.device != device:
        raise ValueError(f"{what}: out must be a contiguous fp32 {list(shape)} tensor on {device}, got "
                         f"{out.dtype} {list(out.shape)} on {out.device}")
    return out


def _on(t, device, what):
    if t.device != device:
        raise ValueError(f"{what} is on {t.device}, the prototypes on {device}")
    return t


def assemble_masks(mask_prototype: torch.Tensor, mask_coeff: torch.Tensor, box: Optional[torch.Tensor],
                   counts: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """assemble_mask for B images: prototypes [B, K, H, W] (any strides), coefficients
    [B, n, K], boxes [B, n, 4] or None, counts [B] int32 on the device (detections per image;
    None = all n) -> masks [B, n, H, W] (rows past counts[b] are left untouched)."""
    proto = _proto_view(mask_prototype, "mask_prototype")
    coeff = _on(_f32(mask_coeff, "mask_coeff"), proto.device, "mask_coeff")
    if proto.dim() != 4 or coeff.dim() != 3:
        raise ValueError(f"assemble_masks: prototypes {tuple(proto.shape)} / coefficients {tuple(coeff.shape)}")
    B, K, H, W = proto.shape
    n = coeff.shape[1]
    if coeff.shape != (B, n, K):
        raise ValueError(f"assemble_masks: coefficients {tuple(coeff.shape)} must be [{B}, n, {K}]")
    bptr = cptr = None
    if box is not None:
        box = _on(_f32(box, "box"), proto.device, "box")
        if box.shape != (B, n, 4):
            raise ValueError(f"assemble_masks: box {tuple(box.shape)} must be [{B}, {n}, 4]")
        bptr = ctypes.c_void_p(box.data_ptr())
    if counts is not None:
        if counts.dtype != torch.int32 or counts.shape != (B,) or counts.device != proto.device \
                or not counts.is_contiguous():
            raise ValueError("assemble_masks: counts must be a contiguous int32 [B] tensor on the prototypes' device")
        cptr = ctypes.c_void_p(counts.data_ptr())
    out = _check_out(out, (B, n, H, W), proto.device, "assemble_masks")
    _lib.check(_lib.lib().tv_yolact_assemble_masks(ctypes.c_void_p(proto.data_ptr()), _lib.strides(proto, 4), B, K, H, W,
                                                   ctypes.c_void_p(coeff.data_ptr()), bptr, cptr, n,
                                                   ctypes.c_void_p(out.data_ptr()), _lib.stream_of(proto.device)),
               "assemble_masks")
    return out


def assemble_masks_indexed(mask_prototype: torch.Tensor, mask_coeff: torch.Tensor, box: Optional[torch.Tensor],
                           det: torch.Tensor, counts: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The node's mask step (yolact_node.py:134) for B images straight from BatchedNMS: prototypes
    [B, K, H, W] (any strides), coefficients [B, A, K] and boxes [B, A, 4] (or None) of every anchor,
    det [B, n] int64 / counts [B] int32 (BatchedNMS outputs) -> masks [B, n, H, W]; rows past
    counts[b] are left untouched."""
    proto = _proto_view(mask_prototype, "mask_prototype")
    coeff = _on(_f32(mask_coeff, "mask_coeff"), proto.device, "mask_coeff")
    if proto.dim() != 4 or coeff.dim() != 3 or det.dim() != 2:
        raise ValueError("assemble_masks_indexed: need prototypes [B, K, H, W], coeff [B, A, K], det [B, n]")
    _on(det, proto.device, "det")
    _on(counts, proto.device, "counts")
    if not det.is_contiguous() or not counts.is_contiguous():
        raise ValueError("assemble_masks_indexed: det and counts must be contiguous")
    B, K, H, W = proto.shape
    A = coeff.shape[1]
    n = det.shape[1]
    if coeff.shape != (B, A, K) or det.shape != (B, n) or det.dtype != torch.int64 or counts.shape != (B,) \
            or counts.dtype != torch.int32:
        raise ValueError("assemble_masks_indexed: need coeff [B, A, K], det [B, n] int64, counts [B] int32")
    bptr = None
    if box is not None:
        box = _on(_f32(box, "box"), proto.device, "box")
        if box.shape != (B, A, 4):
            raise ValueError(f"assemble_masks_indexed: box {tuple(box.shape)} must be [{B}, {A}, 4]")
        bptr = ctypes.c_void_p(box.data_ptr())
    out = _check_out(out, (B, n, H, W), proto.device, "assemble_masks_indexed")
    _lib.check(_lib.lib().tv_yolact_assemble_masks_indexed(
        ctypes.c_void_p(proto.data_ptr()), _lib.strides(proto, 4), B, K, H, W, ctypes.c_void_p(coeff.data_ptr()), bptr,
        A, ctypes.c_void_p(det.data_ptr()), ctypes.c_void_p(counts.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
        _lib.stream_of(proto.device)), "assemble_masks_indexed")
    return out
