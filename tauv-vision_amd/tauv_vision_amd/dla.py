"""Drop-in `DLABackbone` (reference src/tauv_vision/centernet/model/backbones/dla.py:393-416).

Holds the backbone's parameters under the reference's exact key layout (enumerated by the
native planner, csrc/planner.cpp), so `backbone.dla_down.tree_layers.0...` keys load
unchanged. Its compute is fused into `Centernet`'s native forward.
"""
from typing import List

import torch
import torch.nn as nn

from .weights import model_desc, param_layout, seeded_state_dict

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
    stride-2 Tree per height) -> MultiIDAUp -> IDAUpReverse; out_channels = channels[0]."""

    def __init__(self, heights: List[int], channels: List[int], downsamples: int):
        super().__init__()
        self.heights = [int(h) for h in heights]
        self.channels = [int(c) for c in channels]
        self.downsamples = int(downsamples)
        self.out_channels = self.channels[0]
        desc = model_desc(self.heights, self.channels, self.downsamples, [1])
        layout = [(k, s) for k, s in param_layout(desc) if k.startswith("backbone.")]
        populate(self, [(k[len("backbone."):], s) for k, s in layout], seed_layout=layout, prefix="backbone.")
        self._version = [0]
        self.register_load_state_dict_post_hook(lambda module, keys: module._bump())

    def _bump(self):
        self._version[0] += 1

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self._bump()
        return r

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError("tauv_vision_amd fuses the backbone into Centernet's native forward; "
                                  "call Centernet(backbone, object_config)(img)")
