"""Reference state_dict layout (from the native planner) and a seeded synthetic-weight
recipe (no checkpoints travel)."""
import ctypes
import math

import torch

from . import _lib


ARCH_CENTERNET, ARCH_DLA34, ARCH_PROTONET, ARCH_CENTERNET_BACKBONE = 0, 1, 2, 3


def model_desc(heights, channels, downsamples, head_channels, in_h=64, in_w=64, precision="fp32",
               arch=ARCH_CENTERNET):
    if len(channels) != len(heights) + 1:
        raise ValueError("backbone_channels must have len(backbone_heights) + 1 entries")
    if len(heights) > 8 or len(head_channels) > 16:
        raise ValueError("too many backbone levels or heads")
    d = _lib.ModelDesc()
    d.n_levels = len(heights)
    for i, h in enumerate(heights):
        d.heights[i] = int(h)
    for i, c in enumerate(channels):
        d.channels[i] = int(c)
    d.downsamples = int(downsamples)
    d.n_heads = len(head_channels)
    for i, c in enumerate(head_channels):
        d.head_channels[i] = int(c)
    d.in_h, d.in_w = int(in_h), int(in_w)
    if precision not in _lib.DTYPES:
        raise ValueError(f"precision must be one of {sorted(_lib.DTYPES)}")
    d.compute_dtype = _lib.DTYPES[precision]
    d.arch = int(arch)
    return d


def dla34_desc(head_channels, in_h=64, in_w=64, precision="fp32"):
    """CenterpointDLA34 (centerpoint_dla.py:544-578): the DLA-34 structure is fixed."""
    return model_desc([], [16], 2, head_channels, in_h, in_w, precision, arch=ARCH_DLA34)


def protonet_desc(feature_depth, n_prototype_masks, fpn_h=8, fpn_w=8, precision="fp32"):
    """YOLACT Masknet (masknet.py:8-55) over an fpn[0] map of fpn_h x fpn_w."""
    return model_desc([], [feature_depth], 0, [n_prototype_masks], fpn_h, fpn_w, precision, arch=ARCH_PROTONET)


def param_layout(desc):
    """[(key, shape)] in reference registration (state_dict) order."""
    L = _lib.lib()
    n = ctypes.c_int32()
    _lib.check(L.tv_model_param_count(ctypes.byref(desc), ctypes.byref(n)), "param layout")
    out = []
    name = ctypes.create_string_buffer(512)
    shape = (ctypes.c_int64 * 4)()
    nd = ctypes.c_int32()
    for i in range(n.value):
        _lib.check(L.tv_model_param_info(ctypes.byref(desc), i, name, 512, shape, ctypes.byref(nd)), "param info")
        out.append((name.value.decode(), tuple(shape[k] for k in range(nd.value))))
    return out


def geometry(desc):
    L = _lib.lib()
    fl = ctypes.c_double()
    oh, ow, oc, ocp = (ctypes.c_int32() for _ in range(4))
    _lib.check(L.tv_model_geometry(ctypes.byref(desc), ctypes.byref(fl), ctypes.byref(oh), ctypes.byref(ow),
                                   ctypes.byref(oc), ctypes.byref(ocp)), "geometry")
    return dict(flops_per_frame=fl.value, out_h=oh.value, out_w=ow.value, out_channels=oc.value,
                out_cpad=ocp.value)


def seeded_state_dict(layout, conv_seed=0, aux_seed=1):
    """Deterministic weights for a key layout: conv / conv-transpose weights xavier-uniform
    (generator conv_seed); from generator aux_seed in key order: BN gamma U(.75,1.25),
    beta N(0,.1^2), running_mean N(0,.1^2), running_var U(.75,1.25), conv bias U(-.1,.1)."""
    g_conv = torch.Generator().manual_seed(conv_seed)
    g_aux = torch.Generator().manual_seed(aux_seed)
    names = {k for k, _ in layout}
    sd = {}
    for key, shape in layout:
        prefix, leaf = key.rsplit(".", 1)
        bn = (prefix + ".running_mean") in names
        shape = tuple(shape)
        if leaf == "num_batches_tracked":
            sd[key] = torch.tensor(0, dtype=torch.long)
        elif leaf == "running_mean":
            sd[key] = torch.randn(shape, generator=g_aux) * 0.1
        elif leaf == "running_var":
            sd[key] = torch.rand(shape, generator=g_aux) * 0.5 + 0.75
        elif len(shape) == 4:
            bound = math.sqrt(6.0 / ((shape[0] + shape[1]) * shape[2] * shape[3]))
            sd[key] = (torch.rand(shape, generator=g_conv) * 2.0 - 1.0) * bound
        elif bn and leaf == "weight":
            sd[key] = torch.rand(shape, generator=g_aux) * 0.5 + 0.75
        elif bn and leaf == "bias":
            sd[key] = torch.randn(shape, generator=g_aux) * 0.1
        elif leaf == "bias":
            sd[key] = (torch.rand(shape, generator=g_aux) * 2.0 - 1.0) * 0.1
        else:
            raise ValueError(f"unexpected parameter {key} {shape}")
    return sd
