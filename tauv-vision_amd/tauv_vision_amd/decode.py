"""Drop-in decode API (reference src/tauv_vision/centernet/model/decode.py:16-324) on the
native gfx950 kernels: sigmoid + 3x3 peak NMS, exact per-image top-K and the per-detection
gather run on the GPU (csrc/decode.hip) and return one packed record buffer, copied to the
host once — instead of one device sync per scalar (decode.py:211-221).

Differences from the reference:
  * Detection.label / .score are 0-d CPU tensors (the reference's are 0-d tensors on the
    prediction's device, decode.py:212-213); y/x/h/w/depth are Python floats.
  * decode()'s y / x: the reference forms (R * i + offset) / in_h in float64 Python arithmetic
    (decode.py:214-215); the kernel evaluates the same expression in double but the record
    stores it as fp32, so y / x are that float64 value rounded to fp32 (relative error
    <= 6e-8). h / w / depth / score are the reference's fp32 values exactly.
  * top-K ties are broken toward the smaller flat index (torch.topk: unspecified).
  * label / y / x use integer division (== the reference's float32 division, decode.py:271-277,
    while C*H*W < 2^24).
"""
import ctypes
import threading
from dataclasses import dataclass
from math import atan2, pi
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib

REC = 10  # label, score, y, x, h, w, depth, flat index, aux0, aux1


@dataclass
class Detection:
    label: int
    score: float
    y: float
    x: float
    h: float
    w: float
    yaw: Optional[float] = None
    pitch: Optional[float] = None
    roll: Optional[float] = None
    depth: Optional[float] = None


@dataclass
class KeypointDetection:
    label: int
    score: float
    y: float
    x: float
    w: float
    h: float
    depth: float
    keypoints: List[Optional[Tuple[float, float, float]]]
    keypoint_scores: List[Optional[float]]
    keypoint_affinities: List[Optional[Tuple[float, float, float]]]
    cam_t_object: object


def _gpu(t, name):
    return _lib.require_gpu_tensor(t, name)


def _empty_batch_check(B):
    """The reference's heatmap_detect (decode.py:255-279, and so decode / decode_keypoints) flattens
    the heatmap with reshape(B, -1), which torch refuses for an empty batch: the same error here."""
    if B == 0:
        raise RuntimeError("cannot reshape tensor of 0 elements into shape [0, -1] because the unspecified "
                           "dimension size -1 can be any value and is ambiguous")


def heatmap_nms(heatmap: torch.Tensor, kernel_size: int) -> torch.Tensor:
    """decode.py:239-252: keep values equal to their k x k neighbourhood max, else 0."""
    assert kernel_size >= 1 and kernel_size % 2 == 1
    heatmap = _gpu(heatmap, "heatmap")
    B, C, H, W = heatmap.shape
    out = torch.empty((B, C, H, W), dtype=torch.float32, device=heatmap.device)
    if B == 0:  # the reference's max_pool2d returns the empty batch as is
        return out
    _lib.check(_lib.lib().tv_heatmap_nms(ctypes.c_void_p(heatmap.data_ptr()), _lib.strides(heatmap, 4), B, C, H, W,
                                         kernel_size, 0, ctypes.c_void_p(out.data_ptr()),
                                         _lib.stream_of(heatmap.device)), "heatmap_nms")
    return out


def heatmap_detect(heatmap: torch.Tensor, n_detections: int):
    """decode.py:255-279 -> (index [B,K,2] (y, x), label [B,K], score [B,K])."""
    heatmap = _gpu(heatmap, "heatmap")
    B, C, H, W = heatmap.shape
    n = C * H * W
    _empty_batch_check(B)
    if not 1 <= n_detections <= n:
        raise RuntimeError(f"selected index k out of range (k={n_detections}, n={n})")
    flat = heatmap.reshape(B, n).contiguous()
    dev = heatmap.device
    score = torch.empty((B, n_detections), dtype=torch.float32, device=dev)
    idx32 = torch.empty((B, n_detections), dtype=torch.int32, device=dev)
    index = torch.empty((B, n_detections, 2), dtype=torch.int64, device=dev)
    label = torch.empty((B, n_detections), dtype=torch.int64, device=dev)
    L, s = _lib.lib(), _lib.stream_of(dev)
    _lib.check(L.tv_heatmap_topk(ctypes.c_void_p(flat.data_ptr()), B, n, n_detections,
                                 ctypes.c_void_p(score.data_ptr()), ctypes.c_void_p(idx32.data_ptr()), s),
               "heatmap_detect")
    _lib.check(L.tv_index_split(ctypes.c_void_p(idx32.data_ptr()), B, n_detections, H, W,
                                ctypes.c_void_p(index.data_ptr()), ctypes.c_void_p(label.data_ptr()), s),
               "heatmap_detect")
    return index, label, score


class DeviceDecoder:
    """Static-buffer decode for a fixed (B, C, H, W, K): launches sigmoid+NMS, exact top-K
    and the record gather on the current stream into preallocated device buffers, with no
    host synchronisation — so a forward + decode step can be captured in a HIP graph.
    `records` is [B, K, 10] fp32, `counts` [B] int32 (see include/tauv_vision_amd.h)."""

    def __init__(self, B, C, H, W, K, device):
        if not 1 <= K <= C * H * W:
            raise RuntimeError(f"selected index k out of range (k={K}, n={C * H * W})")
        self.shape = (B, C, H, W, K)
        self.device = torch.device(device)
        need = ctypes.c_int64()
        _lib.check(_lib.lib().tv_decode_workspace_size(B, C, H, W, K, ctypes.byref(need)), "decode")
        self.ws_bytes = need.value
        self.ws = torch.zeros(need.value, dtype=torch.uint8, device=self.device)  # counters zero-filled (tv_decode keeps them so)
        # records and counts in one allocation (`packed`): a single D2H copy carries both
        nrec = B * K * REC
        self.packed = torch.empty((nrec + B) * 4, dtype=torch.uint8, device=self.device)
        self.records = self.packed[:nrec * 4].view(torch.float32).view(B, K, REC)
        self.counts = self.packed[nrec * 4:].view(torch.int32)

    def __call__(self, heat, size, offset, depth, mode, ratio, in_h, in_w, thr, aux=None):
        B, C, H, W, K = self.shape
        if tuple(heat.shape) != (B, C, H, W):
            raise ValueError(f"heatmap shape {tuple(heat.shape)} != decoder shape {(B, C, H, W)}")
        dev = self.device

        def ptr_st(t, n, name):
            if t is None:
                return None, None
            t = _gpu(t, name).to(dev)
            return ctypes.c_void_p(t.data_ptr()), _lib.strides(t, n)

        hp, hs = ptr_st(heat, 4, "heatmap")
        sp, ss = ptr_st(size, 4, "size")
        op, os_ = ptr_st(offset, 4, "offset")
        dp, ds = ptr_st(depth, 4, "depth")
        ap, as_ = ptr_st(aux, 5, "keypoint_affinity")
        _lib.check(_lib.lib().tv_decode(hp, hs, sp, ss, op, os_, dp, ds, B, C, H, W, K, mode, ratio, in_h, in_w,
                                        float(thr), ap, as_, ctypes.c_void_p(self.records.data_ptr()),
                                        ctypes.c_void_p(self.counts.data_ptr()), ctypes.c_void_p(self.ws.data_ptr()),
                                        self.ws_bytes, _lib.stream_of(dev)), "decode")
        return self.records, self.counts


_DECODERS = {}  # (device, B, C, H, W, K) -> (DeviceDecoder, pinned host mirror of its packed buffer)
_DECODERS_LOCK = threading.Lock()
_DECODERS_MAX = 8


def _decoder(dev, B, C, H, W, K):
    key = (dev.index, B, C, H, W, K)
    ent = _DECODERS.get(key)
    if ent is None:
        if len(_DECODERS) >= _DECODERS_MAX:
            _DECODERS.pop(next(iter(_DECODERS)))
        dec = DeviceDecoder(B, C, H, W, K, dev)
        ent = (dec, torch.empty(dec.packed.numel(), dtype=torch.uint8, pin_memory=True))
        _DECODERS[key] = ent
    return ent


def _records_many(calls):
    """Run several device decodes back to back on the current stream, each into a cached decoder
    (static workspace and records: no allocation or zero fill per call), copy every packed record
    buffer to pinned host memory and synchronise ONCE. calls: (heat, size, offset, depth, K, mode,
    ratio, in_h, in_w, thr, aux) tuples; returns [(records [B,K,10], counts [B])] host numpy."""
    with _DECODERS_LOCK:
        outs = []
        for heat, size, offset, depth, K, mode, ratio, in_h, in_w, thr, aux in calls:
            heat = _gpu(heat, "heatmap")
            B, C, H, W = heat.shape
            _empty_batch_check(B)
            dec, host = _decoder(heat.device, B, C, H, W, K)
            dec(heat, size, offset, depth, mode, ratio, in_h, in_w, thr, aux)
            host.copy_(dec.packed, non_blocking=True)
            outs.append((host, B, K))
        torch.cuda.current_stream(heat.device).synchronize()
        res = []
        for host, B, K in outs:
            a = host.numpy()
            records = a[:B * K * REC * 4].view(np.float32).reshape(B, K, REC).copy()
            counts = a[B * K * REC * 4:].view(np.int32).copy()
            res.append((records, counts))
        return res


def _records(heat, size, offset, depth, K, mode, ratio, in_h, in_w, thr, aux=None):
    """Run the device decode; returns host numpy records [B,K,10] and counts [B] (one D2H copy)."""
    return _records_many([(heat, size, offset, depth, K, mode, ratio, in_h, in_w, thr, aux)])[0]


def decode_records(prediction, model_config, n_detections: int, score_threshold: float):
    """decode() without the per-detection Python objects: host numpy records [B, K, 10] (label,
    score, y, x, h, w, depth, flat index, -, -; the first counts[b] rows of image b valid) and counts
    [B] int32 — one device decode, one D2H copy, one host synchronisation."""
    return _records(prediction.heatmap, prediction.size, prediction.offset, prediction.depth, n_detections, 0,
                    model_config.downsample_ratio, model_config.in_h, model_config.in_w, score_threshold)


def decode(prediction, model_config, n_detections: int, score_threshold: float) -> List[List[Detection]]:
    """decode.py:179-236."""
    has_depth = prediction.depth is not None
    records, counts = _records(prediction.heatmap, prediction.size, prediction.offset, prediction.depth,
                               n_detections, 0, model_config.downsample_ratio, model_config.in_h, model_config.in_w,
                               score_threshold)
    from .sharding import records_to_detections
    return records_to_detections(records, counts, has_depth)


def decode_keypoints(prediction, model_config, object_config, M_projection, n_detections: int,
                     keypoint_n_detections: int, score_threshold: float, keypoint_score_threshold: float,
                     keypoint_angle_threshold: float) -> List[List[KeypointDetection]]:
    """decode.py:51-176: objects (no offset / ratio, depth = 1/sigmoid) and keypoints from
    the GPU; the greedy affinity-angle matching (decode.py:100-135) runs on the host over
    at most K x K_kp records. `keypoint_angle_threshold` is unused, as in the reference."""
    # both decodes launched back to back, one host synchronisation
    (obj, obj_n), (kp, kp_n) = _records_many([
        (prediction.heatmap, prediction.size, None, prediction.depth, n_detections, 1,
         model_config.downsample_ratio, model_config.in_h, model_config.in_w, score_threshold, None),
        (prediction.keypoint_heatmap, prediction.size, None, None, keypoint_n_detections, 1,
         model_config.downsample_ratio, model_config.in_h, model_config.in_w, keypoint_score_threshold,
         prediction.keypoint_affinity)])
    out = []
    for b in range(obj.shape[0]):
        dets = []
        for r in obj[b, :obj_n[b]]:
            label = int(r[0])
            nk = len(object_config.configs[label].keypoints or [])
            dets.append(KeypointDetection(label=label, score=float(r[1]), y=float(r[2]), x=float(r[3]),
                                          h=float(r[4]), w=float(r[5]),
                                          depth=float(r[6]) if prediction.depth is not None else None,
                                          keypoints=[None] * nk, keypoint_scores=[None] * nk,
                                          keypoint_affinities=[None] * nk, cam_t_object=None))
        for r in kp[b, :kp_n[b]]:
            obj_index, slot = object_config.decode_keypoint_index(int(r[0]))
            cands = [d for d in dets if d.label == obj_index and d.keypoints[slot] is None]
            if not cands:
                continue
            ky, kx = float(r[2]), float(r[3])
            ay, ax = float(r[8]), float(r[9])
            ang = atan2(ay, ax)
            errs = [abs(ang - atan2(ky - d.y, kx - d.x)) for d in cands]
            best = cands[errs.index(min(errs))]
            best.keypoints[slot] = (ky, kx)
            best.keypoint_affinities[slot] = (ay, ax)
            best.keypoint_scores[slot] = float(r[1])
        _solve_poses(dets, model_config, object_config, M_projection)
        out.append(dets)
    return out


def _solve_poses(dets, model_config, object_config, M_projection):
    """decode.py:137-172: PnP for detections with >= 6 matched keypoints (needs OpenCV).
    The reference stores the pose on its last matched detection variable (decode.py:172);
    here it is stored on the detection being solved."""
    for d in dets:
        pts = [(i, k) for i, k in enumerate(d.keypoints) if k is not None]
        if len(pts) < 6:
            continue
        try:
            import cv2
        except ImportError as e:
            raise RuntimeError("decode_keypoints: >= 6 keypoints matched; solvePnP needs OpenCV (cv2)") from e
        img_pts = np.array([[k[1] * model_config.in_w, k[0] * model_config.in_h] for _, k in pts])
        obj_pts = np.array([object_config.configs[d.label].keypoints[i] for i, _ in pts])
        ok, rvec, tvec = cv2.solvePnP(obj_pts, img_pts, M_projection, None, cv2.SOLVEPNP_ITERATIVE)
        if ok:
            rot, _ = cv2.Rodrigues(rvec)
            d.cam_t_object = (rot, tvec)


def angle_get_bins(bin_overlap: float):
    """decode.py:282-288."""
    return ((pi / 2, -bin_overlap / 2, pi + bin_overlap / 2), (-pi / 2, -pi - bin_overlap / 2, bin_overlap / 2))


def angle_decode(predicted_bin: torch.Tensor, predicted_offset: torch.Tensor, theta_range: float,
                 bin_overlap: float) -> torch.Tensor:
    """decode.py:291-316 (not wired into decode() in the reference either)."""
    (c0, _, _), (c1, _, _) = angle_get_bins(bin_overlap)
    p0 = torch.softmax(predicted_bin[..., 0:2], dim=-1)[..., 1]
    p1 = torch.softmax(predicted_bin[..., 2:4], dim=-1)[..., 1]
    a0 = c0 + torch.atan2(predicted_offset[..., 0], predicted_offset[..., 1])
    a1 = c1 + torch.atan2(predicted_offset[..., 2], predicted_offset[..., 3])
    ang = torch.where(p1 > p0, a1, a0) % (2 * pi)
    return ang * (theta_range / (2 * pi))


def depth_decode(prediction: torch.Tensor) -> torch.Tensor:
    """decode.py:319-324."""
    return (1 / torch.sigmoid(prediction)) - 1
