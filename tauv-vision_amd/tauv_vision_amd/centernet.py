"""Drop-in `Centernet` / `Prediction` / `get_head_channels` (reference
src/tauv_vision/centernet/model/centernet.py:13-142) backed by the native MI355X engine.

The module keeps the reference state_dict layout exactly (keys, shapes, order), so
`load_state_dict(torch.load(path))` of a reference checkpoint works unchanged; the
forward pass is one native call (all convolutions as fused MFMA implicit GEMMs, see
csrc/planner.cpp) and returns the reference's `Prediction`, whose tensors are channel
slices of one fp32 NHWC head tensor (same shapes and values, different strides).
"""
import ctypes
import threading
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.nn as nn

from . import _lib
from .config import ObjectConfigSet
from .dla import DLABackbone, populate
from .engine import NativeEngine
from .weights import model_desc, dla34_desc, param_layout

_GRAPH_LOCK = threading.RLock()  # the forward graph cache's launches and captures (all models)


@dataclass
class Prediction:
    heatmap: torch.Tensor                      # [B, n_labels, out_h, out_w]
    keypoint_heatmap: Optional[torch.Tensor]   # [B, n_keypoints, out_h, out_w]
    keypoint_affinity: Optional[torch.Tensor]  # [B, n_keypoints, 2, out_h, out_w]
    size: torch.Tensor                         # [B, out_h, out_w, 2]
    offset: torch.Tensor                       # [B, out_h, out_w, 2]
    roll_bin: Optional[torch.Tensor]           # [B, out_h, out_w, 4]
    roll_offset: Optional[torch.Tensor]
    pitch_bin: Optional[torch.Tensor]
    pitch_offset: Optional[torch.Tensor]
    yaw_bin: Optional[torch.Tensor]
    yaw_offset: Optional[torch.Tensor]
    depth: Optional[torch.Tensor]              # [B, out_h, out_w, 1]


def get_head_channels(object_config: ObjectConfigSet) -> List[int]:
    """centernet.py:114-142: heatmap, [keypoint heatmap, keypoint affinity], size, offset,
    [yaw bin/offset], [pitch bin/offset], [roll bin/offset], [depth]."""
    out = [object_config.n_labels]
    if object_config.train_keypoints:
        out += [object_config.n_keypoints, 2 * object_config.n_keypoints]
    out += [2, 2]
    for flag in (object_config.train_yaw, object_config.train_pitch, object_config.train_roll):
        if flag:
            out += [4, 4]
    if object_config.train_depth:
        out.append(1)
    return out


def prediction_fields(object_config: ObjectConfigSet):
    """Field -> (first channel, channel count), following the reference's pop order
    (centernet.py:77-90): after size/offset it assigns roll, pitch, yaw — although
    get_head_channels created the angle heads yaw, pitch, roll — then depth."""
    widths = get_head_channels(object_config)
    starts = [sum(widths[:i]) for i in range(len(widths))]
    order = ["heatmap"]
    if object_config.train_keypoints:
        order += ["keypoint_heatmap", "keypoint_affinity"]
    order += ["size", "offset"]
    for axis, flag in (("roll", object_config.train_roll), ("pitch", object_config.train_pitch),
                       ("yaw", object_config.train_yaw)):
        if flag:
            order += [f"{axis}_bin", f"{axis}_offset"]
    if object_config.train_depth:
        order.append("depth")
    return {name: (starts[i], widths[i]) for i, name in enumerate(order)}


def prediction_from_nhwc(out: torch.Tensor, object_config: ObjectConfigSet) -> Prediction:
    fields = {f: None for f in Prediction.__dataclass_fields__}
    for name, (s, n) in prediction_fields(object_config).items():
        t = out[..., s:s + n]
        if name in ("heatmap", "keypoint_heatmap"):
            t = t.permute(0, 3, 1, 2)
        elif name == "keypoint_affinity":
            B, H, W, _ = t.shape
            t = t.unflatten(3, (n // 2, 2)).permute(0, 3, 4, 1, 2)
        fields[name] = t
    return Prediction(**fields)


class _NativeModel(nn.Module):
    """Engine cache + the reference forward API shared by Centernet and CenterpointDLA34.
    Subclasses provide `_desc(in_h, in_w)` (the native model description) and `_key()`."""

    def _init_native(self, object_config, precision):
        self.object_config = object_config
        self.head_channels = get_head_channels(object_config)
        if precision not in _lib.DTYPES:
            raise ValueError(f"precision must be one of {sorted(_lib.DTYPES)}")
        self.precision = precision
        self._version = [0]
        self._engines = {}
        # hipGraph replay behind forward()/forward_frames(): a (kind, shape) seen before is replayed
        # from a captured graph instead of launched op by op (set False for eager launches only)
        self.graph_replay = True
        self._graphs = {}
        self.register_load_state_dict_post_hook(lambda module, keys: module.invalidate())

    # -- engine cache ---------------------------------------------------------------
    def invalidate(self):
        self._version[0] += 1
        self._engines = {}
        self._graphs = {}

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self.invalidate()
        return r

    def set_precision(self, precision: str):
        if precision not in _lib.DTYPES:
            raise ValueError(f"precision must be one of {sorted(_lib.DTYPES)}")
        self.precision = precision
        self.invalidate()
        return self

    def _key(self):
        return (self._version[0],)

    def _device_for(self, t: torch.Tensor) -> torch.device:
        if not torch.cuda.is_available():
            raise RuntimeError("tauv_vision_amd needs a gfx950 (MI355X) GPU; no HIP device is visible")
        if t.is_cuda:
            return t.device
        p = next(self.parameters())
        return p.device if p.is_cuda else torch.device("cuda", torch.cuda.current_device())

    def engine(self, device: torch.device, in_h: int, in_w: int) -> NativeEngine:
        key = (device.index if device.index is not None else torch.cuda.current_device(), in_h, in_w,
               self.precision) + self._key()
        eng = self._engines.get(key)
        if eng is None:
            eng = NativeEngine(self._desc(in_h, in_w), self.state_dict(), key[0])
            self._engines = {key: eng}
        return eng

    # -- graph cache ------------------------------------------------------------------
    def _launch(self, eng: NativeEngine, kind: str, x: torch.Tensor) -> torch.Tensor:
        """One engine forward of `x` (kind "f32": normalised NCHW, "u8": NHWC frames) on the caller's
        stream, returning a fresh fp32 NHWC head tensor. Per (caller stream, kind, shape): the first
        call runs eagerly; the second captures the forward once as a hipGraph on a private stream
        (static input / output buffers, the engine workspace keyed to that stream: an eager warm-up
        there, then the capture); every later call copies the input in, replays the graph on the
        caller's stream and returns a copy of the output — so results never alias a later call's,
        as the reference's fresh tensors. Eager when graph_replay is off, while the caller's stream
        is capturing, or if the capture failed (graph_failures). Threads (rospy runs one callback
        thread per camera, centernet_node.py:58-65): launches are enqueued under one lock, so a
        capture never sees another thread's launches; the GPU work of different streams still
        overlaps."""
        fwd = eng.forward_u8 if kind == "u8" else eng.forward
        if x.shape[0] == 0:  # an empty batch: the reference's convolutions return empty outputs
            return eng.alloc_out(0)
        if not self.graph_replay or torch.cuda.is_current_stream_capturing():
            return fwd(x)
        cur = torch.cuda.current_stream(eng.device)
        key = (id(eng), eng.generation, cur.cuda_stream, kind, tuple(x.shape))
        with _GRAPH_LOCK:
            ent = self._graphs.get(key)
            if ent is None:  # first sight: eager (the node's warm-up forward, centernet_node.py:50)
                self._graphs = {k: v for k, v in self._graphs.items() if k[0] == id(eng) and k[1] == eng.generation}
                self._graphs[key] = {"graph": None, "failed": False}
                return fwd(x)
            if ent["failed"]:
                return fwd(x)
            if ent["graph"] is None:
                try:
                    side = torch.cuda.Stream(eng.device)
                    inp = torch.empty_like(x, memory_format=torch.contiguous_format)
                    out = eng.alloc_out(x.shape[0])
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        inp.copy_(x)
                        fwd(inp, out)  # workspace for (side, B) made outside the capture
                        graph = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
                            fwd(inp, out)
                    cur.wait_stream(side)
                    ent.update(graph=graph, stream=side, inp=inp, out=out)
                except RuntimeError as e:  # keep the model usable: this (kind, shape) stays eager
                    import warnings
                    warnings.warn(f"tauv_vision_amd: hipGraph capture failed ({e}); eager launches for {key[3:]}")
                    ent["failed"] = True
                    self.graph_failures = getattr(self, "graph_failures", 0) + 1
                    return fwd(x)
            ent["inp"].copy_(x)
            ent["graph"].replay()
            return ent["out"].clone()

    # -- reference API --------------------------------------------------------------
    def forward(self, img: torch.Tensor) -> Prediction:
        if img.dim() != 4 or img.shape[1] != 3:
            raise ValueError(f"expected img [batch, 3, in_h, in_w], got {tuple(img.shape)}")
        dev = self._device_for(img)
        img = img.to(dev, torch.float32).contiguous()
        eng = self.engine(dev, img.shape[2], img.shape[3])
        return prediction_from_nhwc(self._launch(eng, "f32", img), self.object_config)

    def forward_frames(self, frames: torch.Tensor, size=None) -> Prediction:
        """Raw uint8 RGB camera frames [B, H, W, 3] (or [H, W, 3]) through the node's
        preprocessing (centernet_node.py:90-92): ToTensor -> Resize(size) -> Normalize(ImageNet).
        size = (in_h, in_w) of the model (None: the frames' own size). At the model size the
        resize is the identity and ToTensor + Normalize are fused into the stem kernel; otherwise
        one kernel resizes + normalises (tv_preprocess_u8) into the fp32 forward() input."""
        if frames.dim() == 3:
            frames = frames.unsqueeze(0)
        if frames.dtype != torch.uint8 or frames.shape[-1] != 3:
            raise ValueError("frames must be uint8 [B, H, W, 3]")
        dev = self._device_for(frames)
        frames = frames.to(dev).contiguous()
        in_h, in_w = (frames.shape[1], frames.shape[2]) if size is None else (int(size[0]), int(size[1]))
        eng = self.engine(dev, in_h, in_w)
        if (in_h, in_w) == (frames.shape[1], frames.shape[2]):
            return prediction_from_nhwc(self._launch(eng, "u8", frames), self.object_config)
        return prediction_from_nhwc(self._launch(eng, "f32", preprocess(frames, in_h, in_w)), self.object_config)

    def detect(self, frames: torch.Tensor, model_config, n_detections: int = 100, score_threshold: float = 0.3):
        """detect(frames) == decode(forward(preprocess(frames)), ...): camera frames of any size,
        resized to (model_config.in_h, model_config.in_w) like the node."""
        from .decode import decode
        return decode(self.forward_frames(frames, (model_config.in_h, model_config.in_w)), model_config,
                      n_detections, score_threshold)


class Centernet(_NativeModel):
    """centernet.py:32-92. `precision`: "fp32" (exact-f32 MFMA, parity mode), "fp16" or
    "bf16" (fp32 accumulation; throughput mode)."""

    def __init__(self, backbone: DLABackbone, object_config: ObjectConfigSet, precision: str = "fp32"):
        super().__init__()
        self.backbone = backbone
        self._init_native(object_config, precision)
        desc = model_desc(backbone.heights, backbone.channels, backbone.downsamples, self.head_channels)
        layout = [(k, s) for k, s in param_layout(desc) if k.startswith("heads.")]
        self.heads = nn.Module()
        populate(self.heads, [(k[len("heads."):], s) for k, s in layout], seed_layout=layout, prefix="heads.")

    def _key(self):
        return (self._version[0], self.backbone._version[0])

    def _desc(self, in_h, in_w):
        return model_desc(self.backbone.heights, self.backbone.channels, self.backbone.downsamples,
                          self.head_channels, in_h, in_w, self.precision)


class CenterpointDLA34(_NativeModel):
    """centerpoint_dla.py:544-578: DLASeg('dla34', heads {'0'..'n-1'}, down_ratio 4,
    final_kernel 1, last_level 5, head_conv 256) under `self.model`, so reference checkpoints
    (keys `model.base...`, `model.dla_up...`, `model.ida_up...`, `model.<i>.{0,2}...`) load
    unchanged. The reference constructor downloads ImageNet DLA-34 weights (get_pose_net,
    :534-541); here the parameters start from the seeded recipe and a checkpoint is loaded
    with load_state_dict. DCNv2 runs natively (csrc/dla34.hip + MFMA GEMM over its columns)."""

    def __init__(self, object_config: ObjectConfigSet, precision: str = "fp32"):
        super().__init__()
        self._init_native(object_config, precision)
        layout = param_layout(dla34_desc(self.head_channels))
        self.model = nn.Module()
        populate(self.model, [(k[len("model."):], s) for k, s in layout], seed_layout=layout, prefix="model.")

    def _desc(self, in_h, in_w):
        return dla34_desc(self.head_channels, in_h, in_w, self.precision)


def preprocess(frames: torch.Tensor, in_h: int, in_w: int) -> torch.Tensor:
    """The node's T.ToTensor -> T.Resize((in_h, in_w)) -> T.Normalize(ImageNet)
    (centernet_node.py:90-92) on the GPU: u8 RGB frames [B, H, W, 3] (or [H, W, 3]) at camera
    resolution -> normalised fp32 [B, 3, in_h, in_w] (bilinear, align_corners=False, no antialias:
    torchvision 0.15.2's tensor Resize)."""
    if frames.dim() == 3:
        frames = frames.unsqueeze(0)
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError("frames must be uint8 [B, H, W, 3]")
    if not torch.cuda.is_available():
        raise RuntimeError("tauv_vision_amd needs a gfx950 (MI355X) GPU; no HIP device is visible")
    frames = (frames if frames.is_cuda else frames.cuda()).contiguous()
    B, H, W, _ = frames.shape
    out = torch.empty((B, 3, int(in_h), int(in_w)), dtype=torch.float32, device=frames.device)
    if B == 0:
        return out
    _lib.check(_lib.lib().tv_preprocess_u8(ctypes.c_void_p(frames.data_ptr()), B, H, W, int(in_h), int(in_w),
                                           ctypes.c_void_p(out.data_ptr()), _lib.stream_of(frames.device)),
               "preprocess")
    return out


def initialize_weights(module: nn.Module, excluded_modules=()):
    """centernet.py:103-111 analogue: re-draw every conv/conv-transpose weight xavier-uniform
    and zero its bias (parameter tree leaves with a 4-D weight)."""
    excluded = set()
    for m in excluded_modules:
        excluded.update(id(x) for x in m.modules())
    for sub in module.modules():
        w = sub._parameters.get("weight") if hasattr(sub, "_parameters") else None
        if w is not None and w.dim() == 4 and id(sub) not in excluded:
            with torch.no_grad():
                nn.init.xavier_uniform_(w)
                b = sub._parameters.get("bias")
                if b is not None:
                    b.zero_()
    for m in module.modules():
        if isinstance(m, _NativeModel):
            m.invalidate()
