"""Drop-in YOLACT post-processing (reference src/tauv_vision/yolact/model/):
`get_anchor` (anchors.py:9-41), `box_decode` (boxes.py:55-61), `nms` (nms.py:7-29) and
`assemble_mask` (masks.py:8-21), as called by the YOLACT node (yolact_node.py:128-134).

`box_decode`, `nms` and `assemble_mask` run in the HIP library (csrc/yolact.hip) on the
tensors' GPU; there is no CPU fallback. `get_anchor` builds the per-level anchor constants on
the host exactly like the reference (it is configuration, computed once per FPN level).
"""
from dataclasses import dataclass
from math import sqrt
from typing import Optional, Tuple

import ctypes
import torch

from . import _lib


@dataclass
class YolactConfig:
    """The fields of the reference yolact ModelConfig (config.py:8-40) the post-processing reads."""
    in_w: int
    in_h: int
    anchor_scales: Tuple[int, ...]
    anchor_aspect_ratios: Tuple[float, ...]
    box_variances: Tuple[float, float]


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


def box_decode(box_encoding: torch.Tensor, anchor: torch.Tensor, config) -> torch.Tensor:
    """boxes.py:55-61 on the GPU: [B, A, 4] encodings + [1 or B, A, 4] anchors -> boxes (y, x, h, w)."""
    enc = _f32(box_encoding, "box_encoding")
    anc = _f32(anchor, "anchor").to(enc.device)
    if enc.dim() != 3 or enc.shape[-1] != 4 or anc.dim() != 3 or anc.shape[1:] != enc.shape[1:]:
        raise ValueError(f"box_decode: encodings {tuple(enc.shape)} / anchors {tuple(anc.shape)} mismatch")
    out = torch.empty_like(enc)
    B, A, _ = enc.shape
    _lib.check(_lib.lib().tv_yolact_box_decode(ctypes.c_void_p(enc.data_ptr()), ctypes.c_void_p(anc.data_ptr()), B, A,
                                               anc.shape[0], float(config.box_variances[0]),
                                               float(config.box_variances[1]), ctypes.c_void_p(out.data_ptr()),
                                               _lib.stream_of(enc.device)), "box_decode")
    return out


def nms(classification: torch.Tensor, box: torch.Tensor, top_k: int, iou_threshold: float,
        confidence_threshold: float) -> torch.Tensor:
    """nms.py:7-29 (YOLACT fast NMS, batch 0 only): int64 indices of the kept anchors in
    descending-confidence order. One device->host read of the kept count."""
    cls = _f32(classification, "classification")
    bx = _f32(box, "box").to(cls.device)
    if cls.dim() != 3 or bx.dim() != 3 or bx.shape[-1] != 4 or cls.shape[1] != bx.shape[1]:
        raise ValueError(f"nms: classification {tuple(cls.shape)} / box {tuple(bx.shape)} mismatch")
    A, C1 = cls.shape[1], cls.shape[2]
    K = min(int(top_k), A)
    det = torch.empty((max(K, 1),), dtype=torch.int64, device=cls.device)
    n = torch.empty((1,), dtype=torch.int32, device=cls.device)
    _lib.check(_lib.lib().tv_yolact_fast_nms(ctypes.c_void_p(cls[0].data_ptr()), A, C1, ctypes.c_void_p(bx[0].data_ptr()),
                                             int(top_k), float(iou_threshold), float(confidence_threshold),
                                             ctypes.c_void_p(det.data_ptr()), ctypes.c_void_p(n.data_ptr()),
                                             _lib.stream_of(cls.device)), "nms")
    return det[:int(n.item())]


def assemble_mask(mask_prototype: torch.Tensor, mask_coeff: torch.Tensor,
                  box: Optional[torch.Tensor]) -> torch.Tensor:
    """masks.py:8-21: prototypes [K, H, W], coefficients [n, K], boxes [n, 4] or None -> [n, H, W]."""
    proto = _f32(mask_prototype, "mask_prototype")
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
    _lib.check(_lib.lib().tv_yolact_assemble_mask(ctypes.c_void_p(proto.data_ptr()), K, H, W,
                                                  ctypes.c_void_p(coeff.data_ptr()), bptr, n,
                                                  ctypes.c_void_p(out.data_ptr()), _lib.stream_of(proto.device)),
               "assemble_mask")
    return out
