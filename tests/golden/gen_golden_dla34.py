"""Generate the DLA34 (`CenterpointDLA34`) golden vectors.

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER. It imports the reference module
src/tauv_vision/centernet/model/backbones/centerpoint_dla.py read-only. That file imports
torchvision for `torchvision.ops.DeformConv2d` (centerpoint_dla.py:9,387); torchvision is
absent here, so a stand-in `torchvision.ops.DeformConv2d` module is registered whose
parameters match torchvision 0.15.2's (weight [out, in, 3, 3], then bias [out]) and whose
forward is this repo's own DCNv2 restatement (oracle/ref_dla34.py `deform_conv2d`).
Consequently the goldens pin everything the reference computes around DCNv2 (DLA-34 base,
Trees with ceil-mode max-pool downsampling, Roots, DLAUp/IDAUp with depthwise transposed
convs and pad_to_match, the heads and the Prediction packing) while DCNv2 numerics stay
PARITY UNPINNED.

`CenterpointDLA34.__init__` downloads ImageNet weights (get_pose_net hard-codes
pretrained=True, centerpoint_dla.py:534-541), unavailable offline, so the wrapper is built
around `DLASeg('dla34', heads, pretrained=False, down_ratio=4, final_kernel=1,
last_level=5, head_conv=256)` and its own `forward` is called unchanged.

Weights: the seeded recipe of tests/golden/recipe.py over the reference key list (not
committed; checksums stored). Outputs: .npz inputs/outputs only, no reference source.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_dla34.py
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from recipe import DLA34_CASES, seeded_state_dict, seeded_input  # noqa: E402
from gen_golden import _import_reference, object_config_for, _pack_dets, _pack_kp_dets, _flat_peaks  # noqa: E402
from oracle.ref_dla34 import deform_conv2d  # noqa: E402


class _DeformConv2d(nn.Module):
    """torchvision.ops.DeformConv2d parameter layout; forward = the oracle restatement."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 bias=True):
        super().__init__()
        assert dilation == 1 and groups == 1
        self.stride, self.padding = stride, padding
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, mask, self.weight, self.bias, self.stride, self.padding)


def _import_dla34():
    tv = types.ModuleType("torchvision")
    ops = types.ModuleType("torchvision.ops")
    ops.DeformConv2d = _DeformConv2d
    tv.ops = ops
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.ops", ops)
    rcfg, rnet, rdec, _ = _import_reference()
    from tauv_vision.centernet.model.backbones import centerpoint_dla as rdla34
    return rcfg, rnet, rdec, rdla34


def main():
    rcfg, rnet, rdec, rdla34 = _import_dla34()
    index = {}
    for case in DLA34_CASES:
        name = case["name"]
        torch.manual_seed(0)
        oc = object_config_for(rcfg, case["objects"])
        head_channels = rnet.get_head_channels(oc)
        model = rdla34.CenterpointDLA34.__new__(rdla34.CenterpointDLA34)
        nn.Module.__init__(model)
        model.object_config = oc
        model.model = rdla34.DLASeg("dla34", {str(i): c for i, c in enumerate(head_channels)}, pretrained=False,
                                    down_ratio=4, final_kernel=1, last_level=5, head_conv=256)
        model.eval()
        keys = [(k, list(v.shape)) for k, v in model.state_dict().items()]
        sd = seeded_state_dict(keys)
        model.load_state_dict(sd)
        img = seeded_input(case)
        with torch.no_grad():
            pred = model(img)
        out = {"img_checksum": np.array([float(img.double().sum()), float(img.double().abs().sum())])}
        present = []
        for f in ["heatmap", "keypoint_heatmap", "keypoint_affinity", "size", "offset", "roll_bin", "roll_offset",
                  "pitch_bin", "pitch_offset", "yaw_bin", "yaw_offset", "depth"]:
            t = getattr(pred, f)
            if t is not None:
                out[f] = t.contiguous().numpy()
                present.append(f)
        mc = rcfg.ModelConfig(backbone_heights=[], backbone_channels=[], in_h=case["in_h"], in_w=case["in_w"],
                              downsamples=2, angle_bin_overlap=float(np.pi / 3))
        for thr in (0.05, 0.3):
            out[f"decode_thr{thr}"] = _pack_dets(rdec.decode(pred, mc, 20, thr), 20,
                                                 has_depth=pred.depth is not None)
        out["decode_k100"] = _pack_dets(rdec.decode(pred, mc, 100, 0.0), 100, has_depth=pred.depth is not None)
        out["decode_k100_index"] = _flat_peaks(rdec, pred.heatmap, 100)
        if oc.train_keypoints:
            # the node's call (centernet_node.py:106-116: 10 objects, 50 keypoints) at thresholds
            # low enough for seeded weights to produce matches
            kd = rdec.decode_keypoints(pred, mc, oc, np.eye(3), n_detections=10, keypoint_n_detections=50,
                                       score_threshold=0.05, keypoint_score_threshold=0.05,
                                       keypoint_angle_threshold=0.3)
            out["decode_keypoints"] = _pack_kp_dets(kd, 10, oc)
        out["weight_checksums"] = np.array([[float(v.double().sum()), float(v.double().abs().sum())]
                                            if v.dtype.is_floating_point else [float(v), 0.0]
                                            for v in sd.values()])
        np.savez_compressed(os.path.join(HERE, f"dla34_{name}.npz"), **out)
        index[name] = {"keys": keys, "head_channels": head_channels, "fields": present, "case": case}
        print(f"{name}: {len(keys)} keys, heads {head_channels}, heatmap {tuple(pred.heatmap.shape)}")
    with open(os.path.join(HERE, "models_dla34.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
