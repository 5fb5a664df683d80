"""Oracle (test infrastructure): functional PyTorch-CPU restatement of the reference
CenterNet forward ("R18" map = Centernet + DLABackbone).

Follows, op for op and in the same order (so CPU results are bit-identical):
  * ResidualBlock      dla.py:8-52   (residual branch first, then conv1/bn1/relu, conv2/bn2, +=, relu)
  * Root               dla.py:58-76  (1x1 conv over channel concat, bn, relu)
  * Tree               dla.py:79-135 (height-1 leaf: root(children + [l(x), r(l(x))]);
                                      height>1: tree_r(tree_l(x), children + [xl]))
  * DLADown            dla.py:138-192 (7x7 stem @ full res, `downsamples` s2 blocks, s2 trees)
  * pad_to_match       dla.py:195-209 (F.pad tuple quirk: H excess pads W, W excess pads H)
  * IDAUp              dla.py:212-284, IDAUpReverse dla.py:287-357, MultiIDAUp dla.py:360-390
  * DLABackbone        dla.py:393-416
  * Centernet heads    centernet.py:39-61 (3x3 C->2C + bias, LeakyReLU(0.01), 1x1 2C->n + bias)
  * Prediction packing centernet.py:65-92 (pop order: heatmap, [kp heatmap, kp affinity], size,
                        offset, roll, pitch, yaw, depth — note yaw/pitch/roll are *created* in
                        get_head_channels order yaw,pitch,roll, centernet.py:133-140)
Weights are read from a reference-layout state_dict (same keys).
"""
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F


@dataclass
class PredictionRef:
    heatmap: torch.Tensor
    keypoint_heatmap: Optional[torch.Tensor]
    keypoint_affinity: Optional[torch.Tensor]
    size: torch.Tensor
    offset: torch.Tensor
    roll_bin: Optional[torch.Tensor]
    roll_offset: Optional[torch.Tensor]
    pitch_bin: Optional[torch.Tensor]
    pitch_offset: Optional[torch.Tensor]
    yaw_bin: Optional[torch.Tensor]
    yaw_offset: Optional[torch.Tensor]
    depth: Optional[torch.Tensor]


def head_channels_for(n_labels, n_keypoints, keypoints, yaw, pitch, roll, depth):
    """centernet.py:114-142 head list order."""
    hc = [n_labels]
    if keypoints:
        hc += [n_keypoints, 2 * n_keypoints]
    hc += [2, 2]
    for flag in (yaw, pitch, roll):
        if flag:
            hc += [4, 4]
    if depth:
        hc.append(1)
    return hc


def _conv(sd, p, x, stride=1, padding=0):
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), stride, padding)


def _bn(sd, p, x):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], False, 0.1, 1e-5)


def _block(sd, p, x, stride):
    res = _bn(sd, p + ".bn_residual", _conv(sd, p + ".conv_residual", x, stride))
    y = F.relu(_bn(sd, p + ".bn1", _conv(sd, p + ".conv1", x, stride, 1)))
    y = _bn(sd, p + ".bn2", _conv(sd, p + ".conv2", y, 1, 1))
    y += res
    return F.relu(y)


def _tree(sd, p, x, height, stride, children=None):
    kids = [] if children is None else children
    if height == 1:
        left = _block(sd, p + ".tree_l", x, stride)
        right = _block(sd, p + ".tree_r", left, 1)
        cat = torch.cat(kids + [left, right], 1)
        return F.relu(_bn(sd, p + ".root.bn", _conv(sd, p + ".root.conv", cat)))
    left = _tree(sd, p + ".tree_l", x, height - 1, stride)
    return _tree(sd, p + ".tree_r", left, height - 1, 1, kids + [left])


def pad_to_match(feature, shape):
    """dla.py:195-209, quirk preserved: the 4-tuple is (above, below, left, right) but
    F.pad reads it as (W_left, W_right, H_top, H_bottom)."""
    if feature.shape == shape:
        return feature
    fh, fw = feature.shape[2], feature.shape[3]
    th, tw = shape[2], shape[3]
    above = max(0, (fh - th) // 2)
    below = max(0, th - fh - above)
    left = max(0, (fw - tw) // 2)
    right = max(0, tw - fw - left)
    return F.pad(feature, (above, below, left, right))[:, :, :th, :tw]


def _proj(sd, p, x):
    return F.relu(_bn(sd, p + ".1", _conv(sd, p + ".0", x, 1, 1)))


def _ida_up(sd, p, feats):
    n = len(feats) - 1
    cur = feats[-1]
    outs = []
    for i in reversed(range(n)):
        up = sd[f"{p}.upsample_layers.{i}.weight"]
        s = up.shape[2]
        u = F.conv_transpose2d(_proj(sd, f"{p}.projection_layers.{i}", cur), up,
                               sd[f"{p}.upsample_layers.{i}.bias"], stride=s)
        cur = _proj(sd, f"{p}.output_layers.{i}", feats[i] + pad_to_match(u, feats[i].shape))
        outs.append(cur)
    return outs[::-1]


def _ida_up_reverse(sd, p, feats):
    cur = feats[0]
    for i in range(len(feats) - 1):
        up = sd[f"{p}.upsample_layers.{i}.weight"]
        s = up.shape[2]
        u = F.conv_transpose2d(_proj(sd, f"{p}.projection_layers.{i}", feats[i + 1]), up,
                               sd[f"{p}.upsample_layers.{i}.bias"], stride=s)
        cur = _proj(sd, f"{p}.output_layers.{i}", cur + pad_to_match(u, cur.shape))
    return cur


def backbone_forward(sd, img, heights, downsamples, prefix="backbone"):
    p = prefix + ".dla_down"
    x = F.relu(_bn(sd, p + ".projection_layer.1", _conv(sd, p + ".projection_layer.0", img, 1, 3)))
    for i in range(downsamples):
        x = _block(sd, f"{p}.block_layers.{i}", x, 2)
    feats = [x]
    for i, h in enumerate(heights):
        x = _tree(sd, f"{p}.tree_layers.{i}", x, h, 2)
        feats.append(x)
    # MultiIDAUp: IDAUp over a shrinking feature list, keep the last output of each
    collected = []
    for i in range(len(feats) - 1):
        feats = _ida_up(sd, f"{prefix}.multi_ida_up.ida_up_layers.{i}", feats)
        collected.append(feats[-1])
    collected = collected[::-1]
    return _ida_up_reverse(sd, prefix + ".ida_up_reverse", collected)


def centernet_forward(sd, img, heights, downsamples, flags):
    """flags: dict(keypoints, yaw, pitch, roll, depth) as in ObjectConfigSet.train_*."""
    feat = backbone_forward(sd, img, heights, downsamples)
    outs = []
    i = 0
    while f"heads.{i}.0.weight" in sd:
        h = F.leaky_relu(F.conv2d(feat, sd[f"heads.{i}.0.weight"], sd[f"heads.{i}.0.bias"], 1, 1))
        outs.append(F.conv2d(h, sd[f"heads.{i}.2.weight"], sd[f"heads.{i}.2.bias"]))
        i += 1

    def nhwc(t):
        return t.permute(0, 2, 3, 1)

    heat = outs.pop(0)
    kh = ka = None
    if flags.get("keypoints"):
        kh = outs.pop(0)
        t = outs.pop(0)
        ka = t.reshape(t.size(0), t.size(1) // 2, 2, t.size(2), t.size(3))
    size = nhwc(outs.pop(0))
    offset = nhwc(outs.pop(0))
    ang = {}
    for name in ("roll", "pitch", "yaw"):
        if flags.get(name):
            ang[name] = (nhwc(outs.pop(0)), nhwc(outs.pop(0)))
        else:
            ang[name] = (None, None)
    depth = nhwc(outs.pop(0)) if flags.get("depth") else None
    return PredictionRef(heatmap=heat, keypoint_heatmap=kh, keypoint_affinity=ka, size=size,
                         offset=offset, roll_bin=ang["roll"][0], roll_offset=ang["roll"][1],
                         pitch_bin=ang["pitch"][0], pitch_offset=ang["pitch"][1],
                         yaw_bin=ang["yaw"][0], yaw_offset=ang["yaw"][1], depth=depth)
