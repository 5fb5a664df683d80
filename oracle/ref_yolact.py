"""Oracle (test infrastructure): PyTorch-CPU restatement of the reference's YOLACT
post-processing (src/tauv_vision/yolact/model/), pinned by tests/golden/gen_golden_yolact.py
(goldens made by importing the reference modules, which import cleanly here).

  get_anchor     anchors.py:9-41   cell-centre anchors per FPN level, one block per aspect ratio
  box_decode     boxes.py:55-61    c = a_c + e_c * v0 * a_hw ; hw = a_hw * exp(e_hw * v1)
  iou_matrix     boxes.py:64-85    corners (boxes.py:14-26), clamped intersection, union = areas - inter
  nms            nms.py:7-29       softmax, max over non-background, sort desc, top_k, triu IoU,
                                   column max, keep (iou_max <= thr) & (conf >= cthr); batch 0 only
  assemble_mask  masks.py:8-21     per detection sigmoid(sum_k c_k P_k) x box_to_mask (boxes.py:88-103)
  box_encode     boxes.py:45-53    e_c = (b_c - a_c) / (v0 * a_hw) ; e_hw = log(b_hw / a_hw) / v1
  masknet        masknet.py:8-55   protonet: [3x3 conv + LeakyReLU, ConvTranspose2d(3, s2, p1) to 2x
                                   size + LeakyReLU] x 2, 3x3 conv + LeakyReLU, 1x1 conv + LeakyReLU
"""
from math import sqrt

import torch
import torch.nn.functional as F


def get_anchor(fpn_i, fpn_size, anchor_scales, anchor_aspect_ratios, in_h, in_w):
    hh, ww = fpn_size
    ys = ((torch.arange(0, hh) + 0.5) / hh).view(hh, 1).expand(hh, ww).reshape(1, -1)
    xs = ((torch.arange(0, ww) + 0.5) / ww).view(1, ww).expand(hh, ww).reshape(1, -1)
    n = len(anchor_aspect_ratios)
    ys, xs = ys.repeat(1, n), xs.repeat(1, n)
    base = anchor_scales[fpn_i] / ((in_h + in_w) / 2)
    h = torch.cat([torch.full((1, hh * ww), base * sqrt(a)) for a in anchor_aspect_ratios], 1)
    w = torch.cat([torch.full((1, hh * ww), base / sqrt(a)) for a in anchor_aspect_ratios], 1)
    return torch.stack([ys, xs, h, w], 2)


def box_decode(enc, anchor, variances):
    c = anchor[..., :2] + enc[..., :2] * variances[0] * anchor[..., 2:]
    hw = anchor[..., 2:] * torch.exp(enc[..., 2:] * variances[1])
    return torch.cat([c, hw], -1)


def box_encode(box, anchor, variances):
    c = box[..., :2] - anchor[..., :2]
    c = c / (variances[0] * anchor[..., 2:])
    hw = torch.log(box[..., 2:] / anchor[..., 2:]) / variances[1]
    return torch.cat([c, hw], -1)


def masknet(sd, x):
    """Masknet.forward (masknet.py:44-55) over fpn[0] x [B, F, H, W] with state_dict `sd`.
    ConvTranspose2d(3, stride 2, padding 1) called with output_size = 2x -> output_padding 1."""
    def conv(t, name, pad):
        return F.leaky_relu(F.conv2d(t, sd[name + ".weight"], sd[name + ".bias"], padding=pad))

    def up(t, name):
        return F.leaky_relu(F.conv_transpose2d(t, sd[name + ".weight"], sd[name + ".bias"], stride=2, padding=1,
                                               output_padding=1))

    x = up(conv(x, "_layers_1.0.0", 1), "_upsample_layer_1")
    x = up(conv(x, "_layers_2.0.0", 1), "_upsample_layer_2")
    x = conv(x, "_layers_3.0.0", 1)
    return conv(x, "_output_layer", 0)


def _corners(b):
    return torch.stack([b[..., 0] - b[..., 2] / 2, b[..., 1] - b[..., 3] / 2,
                        b[..., 0] + b[..., 2] / 2, b[..., 1] + b[..., 3] / 2], -1)


def iou_matrix(a, b):
    ca, cb = _corners(a), _corners(b)
    y0 = torch.max(ca[..., 0:1], cb[..., 0].unsqueeze(-2))
    x0 = torch.max(ca[..., 1:2], cb[..., 1].unsqueeze(-2))
    y1 = torch.min(ca[..., 2:3], cb[..., 2].unsqueeze(-2))
    x1 = torch.min(ca[..., 3:4], cb[..., 3].unsqueeze(-2))
    inter = (y1 - y0).clamp(min=0) * (x1 - x0).clamp(min=0)
    area_a = (a[..., 2] * a[..., 3]).unsqueeze(-1)
    area_b = (b[..., 2] * b[..., 3]).unsqueeze(-2)
    return inter / ((area_a + area_b) - inter)


def nms(classification, box, top_k, iou_threshold, confidence_threshold):
    conf = F.softmax(classification[0], dim=-1)[:, 1:].max(dim=-1).values
    conf, order = conf.sort(descending=True)
    order, conf = order[:top_k], conf[:top_k]
    b = box[0, order]
    iou_max = torch.triu(iou_matrix(b, b), diagonal=1).max(dim=0).values
    return order[(iou_max <= iou_threshold) & (conf >= confidence_threshold)]


def assemble_mask(proto, coeff, box):
    K, H, W = proto.shape
    out = torch.zeros(coeff.shape[0], H, W)
    yy = torch.arange(H, dtype=torch.float).view(H, 1)
    xx = torch.arange(W, dtype=torch.float).view(1, W)
    for i in range(coeff.shape[0]):
        m = torch.sigmoid((coeff[i].view(K, 1, 1) * proto).sum(0))
        if box is not None:
            bb = box[i] * torch.tensor([H, W, H, W], dtype=torch.float)
            inside = ((xx >= bb[1] - bb[3] / 2) & (xx <= bb[1] + bb[3] / 2) &
                      (yy >= bb[0] - bb[2] / 2) & (yy <= bb[0] + bb[2] / 2))
            m = m * inside.float()
        out[i] = m
    return out
