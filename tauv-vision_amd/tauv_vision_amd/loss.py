"""Training targets of the CenterNet loss on the GPU — reference
src/tauv_vision/centernet/model/loss.py:31-135 (generate_heatmap, generate_keypoint_heatmap,
out_index_for_position), same names, argument meaning and output layout, backed by
tv_train_heatmap / tv_train_keypoint_targets (csrc/targets.hip). The losses themselves
(focal / L1 / angle, loss.py:178-376) stay out of scope (training).

`truth` is the reference's PoseSample (datasets/load/pose_dataset.py:25-41) or this module's
PoseSample with the fields the generators read; its tensors may be on the host (they are
moved to the GPU). The outputs are fp32 device tensors.
"""
import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib


@dataclass
class PoseSample:
    """The fields of the reference's PoseSample (pose_dataset.py:25-41) the targets read."""
    valid: torch.Tensor                           # [B, n_objects] bool
    label: torch.Tensor                           # [B, n_objects] int
    center: torch.Tensor                          # [B, n_objects, 2] (y, x) normalised
    keypoint_valid: Optional[torch.Tensor] = None         # [B, n_keypoint_instances] bool
    keypoint_label: Optional[torch.Tensor] = None         # [B, n_keypoint_instances] int
    keypoint_center: Optional[torch.Tensor] = None        # [B, n_keypoint_instances, 2]
    keypoint_object_index: Optional[torch.Tensor] = None  # [B, n_keypoint_instances] int
    img: Optional[torch.Tensor] = None
    size: Optional[torch.Tensor] = None


def _device(t):
    if not torch.cuda.is_available():
        raise RuntimeError("tauv_vision_amd needs a gfx950 (MI355X) GPU; no HIP device is visible")
    return t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())


def _as(t, dtype, dev):
    return t.to(device=dev, dtype=dtype).contiguous()


def _check_index(idx, valid, bound, what):
    """The reference indexes with these values (heatmap[sample_i, label]): out of range raises."""
    if idx.numel() and bool(((idx < -bound) | (idx >= bound))[valid].any()):
        raise IndexError(f"{what} out of range for {bound} planes")


def _out_shape(model_config):
    """The kernels derive the target grid as in_h // downsample_ratio x in_w // downsample_ratio
    (the reference ModelConfig's out_h / out_w, config.py:24-30) and write it through raw pointers:
    a duck-typed config whose out_h / out_w disagree would be written out of bounds."""
    r = int(model_config.downsample_ratio)
    if r < 1:
        raise ValueError(f"downsample_ratio must be >= 1, got {r}")
    H, W = int(model_config.in_h) // r, int(model_config.in_w) // r
    if (int(model_config.out_h), int(model_config.out_w)) != (H, W):
        raise ValueError(f"model_config.out_h/out_w = ({model_config.out_h}, {model_config.out_w}) but the "
                         f"targets grid is in_h // downsample_ratio x in_w // downsample_ratio = ({H}, {W})")
    return H, W


def generate_heatmap(truth, model_config, train_config, object_config) -> torch.Tensor:
    """loss.py:31-72 -> [B, n_labels, out_h, out_w] fp32 on the GPU."""
    H, W = _out_shape(model_config)
    dev = _device(truth.valid)
    B, n_obj = truth.valid.shape
    L = object_config.n_labels
    valid = _as(truth.valid, torch.uint8, dev)
    label = _as(truth.label, torch.int64, dev)
    center = _as(truth.center, torch.float32, dev)
    _check_index(label, valid.bool(), L, "label")
    label = torch.where(label < 0, label + L, label)
    out = torch.empty((B, L, H, W), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().tv_train_heatmap(
        ctypes.c_void_p(valid.data_ptr()), ctypes.c_void_p(label.data_ptr()), ctypes.c_void_p(center.data_ptr()),
        B, n_obj, L, model_config.in_h, model_config.in_w, model_config.downsample_ratio,
        float(train_config.keypoint_heatmap_sigma), ctypes.c_void_p(out.data_ptr()), _lib.stream_of(dev)),
        "generate_heatmap")
    return out


def generate_keypoint_heatmap(truth, model_config, train_config, object_config):
    """loss.py:75-135 -> (heatmap, affinity_weight [B, n_keypoints, out_h, out_w],
    affinity [B, n_keypoints, 2, out_h, out_w]) fp32 on the GPU."""
    H, W = _out_shape(model_config)
    dev = _device(truth.keypoint_valid)
    B, n_inst = truth.keypoint_valid.shape
    n_obj = truth.center.shape[1]
    K = object_config.n_keypoints
    kvalid = _as(truth.keypoint_valid, torch.uint8, dev)
    klabel = _as(truth.keypoint_label, torch.int64, dev)
    kcenter = _as(truth.keypoint_center, torch.float32, dev)
    kobj = _as(truth.keypoint_object_index, torch.int64, dev)
    center = _as(truth.center, torch.float32, dev)
    _check_index(klabel, kvalid.bool(), K, "keypoint_label")
    _check_index(kobj, kvalid.bool(), n_obj, "keypoint_object_index")
    klabel = torch.where(klabel < 0, klabel + K, klabel)
    kobj = torch.where(kobj < 0, kobj + n_obj, kobj)
    heat = torch.empty((B, K, H, W), dtype=torch.float32, device=dev)
    aw = torch.empty_like(heat)
    aff = torch.empty((B, K, 2, H, W), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().tv_train_keypoint_targets(
        ctypes.c_void_p(kvalid.data_ptr()), ctypes.c_void_p(klabel.data_ptr()), ctypes.c_void_p(kcenter.data_ptr()),
        ctypes.c_void_p(kobj.data_ptr()), ctypes.c_void_p(center.data_ptr()), B, n_inst, n_obj, K,
        model_config.in_h, model_config.in_w, model_config.downsample_ratio,
        float(train_config.keypoint_heatmap_sigma), float(train_config.keypoint_affinity_sigma),
        ctypes.c_void_p(heat.data_ptr()), ctypes.c_void_p(aw.data_ptr()), ctypes.c_void_p(aff.data_ptr()),
        _lib.stream_of(dev)), "generate_keypoint_heatmap")
    return heat, aw, aff


def out_index_for_position(position: torch.Tensor, model_config) -> torch.Tensor:
    """loss.py:131-135: output cell (y, x) of normalised positions [B, n, 2] (a two-op
    elementwise map, left to torch on the positions' device)."""
    return torch.stack((
        torch.clamp(((position[:, :, 0] * model_config.in_h) / model_config.downsample_ratio).to(torch.long), 0,
                    model_config.out_h - 1),
        torch.clamp(((position[:, :, 1] * model_config.in_w) / model_config.downsample_ratio).to(torch.long), 0,
                    model_config.out_w - 1),
    ), dim=-1)
