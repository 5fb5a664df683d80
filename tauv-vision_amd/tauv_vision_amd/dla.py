"""Drop-in `DLABackbone` (reference src/tauv_vision/centernet/model/backbones/dla.py:393-416).

Holds the backbone's parameters under the reference's exact key layout (enumerated by the
native planner, csrc/planner.cpp), so `backbone.dla_down.tree_layers.0...` keys load
unchanged. Inside Centernet its compute is fused into the network's native forward; on its
own it runs the backbone-only native plan.
"""
from typing import List

import torch
import torch.nn as nn

from .weights import ARCH_CENTERNET_BACKBONE, model_desc, param_layout, seeded_state_dict

_BUFFERS = ("running_mean", "running_var", "num_batches_tracked")


def populate(root: nn.Module, layout, seed_layout=None, prefix=""):
    """Create the nested module/parameter tree for `layout` [(key, shape)] under `root`,
    initialised with the seeded recipe (drawn over `seed_layout`, keys prefixed)."""
    init = seeded_state_dict(seed_layout if seed_layout is not None else layout)
    for key, shape in layout:
        *path, leaf = key.split(".")
        mod = root
        for part in path:
            if part not in mod._modules:
                mod.add_module(part, nn.Module())
            mod = mod._modules[part]
        value = init[prefix + key].clone()
        if leaf in _BUFFERS:
            mod.register_buffer(leaf, value)
        else:
            mod.register_parameter(leaf, nn.Parameter(value, requires_grad=False))


class DLABackbone(nn.Module):
    """dla.py:393-416: DLADown (7x7 stem, `downsamples` stride-2 residual blocks, one
    stride-2 Tree per height) -> MultiIDAUp -> IDAUpReverse; out_channels = channels[0].

    Inside `Centernet` the backbone's compute is fused into the network's native forward (its
    output feeds the heads without leaving HBM). Called on its own, `forward(img)` runs the
    backbone-only native plan (TV_ARCH_CENTERNET_BACKBONE) and returns the reference's
    [B, channels[0], in_h / 2^downsamples, in_w / 2^downsamples] fp32 feature map — a permuted
    view of the native NHWC output (same shape and values, channel-last strides). `precision`
    as for Centernet ("fp32" parity mode by default)."""

    def __init__(self, heights: List[int], channels: List[int], downsamples: int, precision: str = "fp32"):
        super().__init__()
        self.heights = [int(h) for h in heights]
        self.channels = [int(c) for c in channels]
        self.downsamples = int(downsamples)
        self.out_channels = self.channels[0]
        self.precision = precision
        desc = model_desc(self.heights, self.channels, self.downsamples, [1])
        layout = [(k, s) for k, s in param_layout(desc) if k.startswith("backbone.")]
        populate(self, [(k[len("backbone."):], s) for k, s in layout], seed_layout=layout, prefix="backbone.")
        self._version = [0]
        self._engines = {}
        self.register_load_state_dict_post_hook(lambda module, keys: module._bump())

    def _bump(self):
        self._version[0] += 1
        self._engines = {}

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self._bump()
        return r

    def engine(self, device: torch.device, in_h: int, in_w: int):
        from .engine import NativeEngine
        key = (device.index if device.index is not None else torch.cuda.current_device(), in_h, in_w,
               self.precision, self._version[0])
        eng = self._engines.get(key)
        if eng is None:
            desc = model_desc(self.heights, self.channels, self.downsamples, [1], in_h, in_w, self.precision,
                              arch=ARCH_CENTERNET_BACKBONE)
            sd = {"backbone." + k: v for k, v in self.state_dict().items()}
            eng = NativeEngine(desc, sd, key[0])
            self._engines = {key: eng}
        return eng

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        if img.dim() != 4 or img.shape[1] != 3:
            raise ValueError(f"expected img [batch, 3, in_h, in_w], got {tuple(img.shape)}")
        if not torch.cuda.is_available():
            raise RuntimeError("tauv_vision_amd needs a gfx950 (MI355X) GPU; no HIP device is visible")
        dev = img.device if img.is_cuda else torch.device("cuda", torch.cuda.current_device())
        img = img.to(dev, torch.float32).contiguous()
        out = self.engine(dev, img.shape[2], img.shape[3]).forward(img)
        return out.permute(0, 3, 1, 2)
