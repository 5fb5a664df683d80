"""Oracle (test infrastructure): PyTorch-CPU restatement of the reference's training-target
generation (src/tauv_vision/centernet/model/loss.py), op for op in the reference's order and
dtypes, pinned to fixtures the reference itself produced (tests/golden/gen_golden_targets.py):

  generate_heatmap           loss.py:31-72   per sample, per valid object: center cell
                                             (floor(c * in / ratio)), Gaussian with the
                                             *keypoint* heatmap sigma (clamped to >= 0.1, :59-63),
                                             max into the object's label plane; nan_to_num
  generate_keypoint_heatmap  loss.py:75-135  per valid keypoint instance, in order: heatmap and
                                             affinity weight Gaussians (max), unit displacement
                                             from the owning object's center to every cell taken
                                             where the distance is strictly smaller than the
                                             running minimum (earliest instance wins ties);
                                             nan_to_num of all three outputs
  out_index_for_position     loss.py:131-135 clamp((p * in) / ratio -> long)

`truth` is any object with the PoseSample fields used here (valid, label, center,
keypoint_valid, keypoint_label, keypoint_center, keypoint_object_index).
"""
from math import floor

import torch


def _cell(c, in_size, ratio):
    # loss.py:52-53 / :103-104: floor(0-d float32 tensor * int / int)
    return floor(c * in_size / ratio)


def generate_heatmap(truth, mc, tc, n_labels):
    B, n_obj = truth.valid.shape
    out_h, out_w = mc.out_h, mc.out_w
    heat = torch.zeros((B, n_labels, out_h, out_w), dtype=torch.float32)
    y, x = torch.meshgrid(torch.arange(0, out_h), torch.arange(0, out_w), indexing="ij")
    for b in range(B):
        for o in range(n_obj):
            if not truth.valid[b, o]:
                continue
            cy = _cell(truth.center[b, o, 0], mc.in_h, mc.downsample_ratio)
            cx = _cell(truth.center[b, o, 1], mc.in_w, mc.downsample_ratio)
            sigma = tc.keypoint_heatmap_sigma
            if sigma < 0.1:
                sigma = 0.1
            lab = truth.label[b, o]
            heat[b, lab] = torch.maximum(heat[b, lab], torch.exp(-((x - cx) ** 2 + (y - cy) ** 2) / (2 * sigma ** 2)))
    return torch.nan_to_num(heat)


def generate_keypoint_heatmap(truth, mc, tc, n_keypoints):
    B, n_inst = truth.keypoint_valid.shape
    out_h, out_w = mc.out_h, mc.out_w
    heat = torch.zeros((B, n_keypoints, out_h, out_w), dtype=torch.float32)
    aw = torch.zeros((B, n_keypoints, out_h, out_w), dtype=torch.float32)
    aff = torch.zeros((B, n_keypoints, 2, out_h, out_w), dtype=torch.float32)
    dist = torch.full((B, n_keypoints, out_h, out_w), fill_value=torch.inf, dtype=torch.float32)
    y, x = torch.meshgrid(torch.arange(0, out_h), torch.arange(0, out_w), indexing="ij")
    for b in range(B):
        for i in range(n_inst):
            if not truth.keypoint_valid[b, i]:
                continue
            k = truth.keypoint_label[b, i]
            cy = _cell(truth.keypoint_center[b, i, 0], mc.in_h, mc.downsample_ratio)
            cx = _cell(truth.keypoint_center[b, i, 1], mc.in_w, mc.downsample_ratio)
            d2 = (x - cx) ** 2 + (y - cy) ** 2
            heat[b, k] = torch.maximum(heat[b, k], torch.exp(-d2 / (2 * tc.keypoint_heatmap_sigma ** 2)))
            aw[b, k] = torch.maximum(aw[b, k], torch.exp(-d2 / (2 * tc.keypoint_affinity_sigma ** 2)))
            disp = torch.stack((y / mc.out_h, x / mc.out_w), dim=0) - \
                truth.center[b, truth.keypoint_object_index[b, i]].unsqueeze(1).unsqueeze(2)
            disp = torch.nan_to_num(disp, 0)
            dd = torch.nan_to_num(torch.sqrt(disp[0] ** 2 + disp[1] ** 2), 1)
            a = disp / dd
            aff[b, k] = torch.where(dd < dist[b, k], a, aff[b, k])
            dist[b, k] = torch.min(dist[b, k], dd)
    return torch.nan_to_num(heat), torch.nan_to_num(aw), torch.nan_to_num(aff)


def out_index_for_position(position, mc):
    return torch.stack((
        torch.clamp(((position[:, :, 0] * mc.in_h) / mc.downsample_ratio).to(torch.long), 0, mc.out_h - 1),
        torch.clamp(((position[:, :, 1] * mc.in_w) / mc.downsample_ratio).to(torch.long), 0, mc.out_w - 1),
    ), dim=-1)
