"""Oracle (test infrastructure): PyTorch-CPU restatement of the reference decode path.

  heatmap_nms        decode.py:239-252  max_pool2d(k, s=1, p=(k-1)/2) then (max == h) * h
  heatmap_detect     decode.py:255-279  flat topk over C*H*W; label/y/x by float32 true
                                        division + truncation, exactly as the reference
  decode             decode.py:179-236  sigmoid -> nms(3) -> topk -> per-detection host loop,
                                        stop at first score < threshold; y/x use
                                        (R*i + offset)/in_{h,w} in Python float arithmetic
  decode_keypoints   decode.py:51-176   objects without offset/ratio, depth = 1/sigmoid(d);
                                        keypoints greedily matched by affinity angle. The PnP
                                        stage (>= 6 keypoints, cv2) is not restated: every
                                        config here has <= 1 keypoint per object.
  depth_decode       decode.py:319-324
Records are returned as plain float tuples (the reference's Detection.label/score are
0-d tensors; only their values are compared).
"""
from math import atan2

import torch
import torch.nn.functional as F


def heatmap_nms(heatmap, kernel_size):
    assert kernel_size >= 1 and kernel_size % 2 == 1
    hmax = F.max_pool2d(heatmap, (kernel_size, kernel_size), stride=1, padding=(kernel_size - 1) // 2)
    return (hmax == heatmap).float() * heatmap


def heatmap_detect(heatmap, n_detections):
    B, C, H, W = heatmap.shape
    score, flat = torch.topk(heatmap.reshape(B, -1), n_detections)
    label = (flat / (H * W)).to(torch.long)
    rem = (flat % (H * W)).to(torch.long)
    index = torch.stack(((rem / W).to(torch.long), (rem % W).to(torch.long)), dim=-1)
    return index, label, score


def depth_decode(prediction):
    return (1 / torch.sigmoid(prediction)) - 1


def decode(prediction, in_h, in_w, downsamples, n_detections, score_threshold):
    """Returns [[(label, score, y, x, h, w, depth_or_None)]]."""
    ratio = 2 ** downsamples
    peaks = heatmap_nms(torch.sigmoid(prediction.heatmap), 3)
    index, label, score = heatmap_detect(peaks, n_detections)
    depth = depth_decode(prediction.depth) if prediction.depth is not None else None
    out = []
    for b in range(index.shape[0]):
        dets = []
        for k in range(n_detections):
            if score[b, k] < score_threshold:
                break
            iy, ix = index[b, k, 0], index[b, k, 1]
            y = (ratio * float(iy) + float(prediction.offset[b, iy, ix, 0])) / in_h
            x = (ratio * float(ix) + float(prediction.offset[b, iy, ix, 1])) / in_w
            h = float(prediction.size[b, iy, ix, 0])
            w = float(prediction.size[b, iy, ix, 1])
            d = float(depth[b, iy, ix, 0]) if depth is not None else None
            dets.append((int(label[b, k]), float(score[b, k]), y, x, h, w, d))
        out.append(dets)
    return out


def decode_keypoints(prediction, out_h, out_w, keypoint_owner, n_detections, keypoint_n_detections,
                     score_threshold, keypoint_score_threshold):
    """keypoint_owner: list mapping flat keypoint index -> (object label, keypoint slot)
    (ObjectConfigSet.decode_keypoint_index, config.py:129-144,192-193); n_kp_per_label[l]
    is implied by it. Returns per image a list of dicts."""
    peaks = heatmap_nms(torch.sigmoid(prediction.heatmap), 3)
    index, label, score = heatmap_detect(peaks, n_detections)
    kpeaks = heatmap_nms(torch.sigmoid(prediction.keypoint_heatmap), 3)
    kindex, klabel, kscore = heatmap_detect(kpeaks, keypoint_n_detections)
    depth = 1 / torch.sigmoid(prediction.depth) if prediction.depth is not None else None
    n_slots = {}
    for lab, slot in keypoint_owner:
        n_slots[lab] = max(n_slots.get(lab, 0), slot + 1)
    out = []
    for b in range(index.shape[0]):
        dets = []
        for k in range(n_detections):
            if score[b, k] < score_threshold:
                break
            lab = int(label[b, k])
            iy, ix = index[b, k, 0], index[b, k, 1]
            nk = n_slots.get(lab, 0)
            dets.append(dict(
                label=lab, score=float(score[b, k]),
                y=float(iy / out_h), x=float(ix / out_w),
                h=float(prediction.size[b, iy, ix, 0]), w=float(prediction.size[b, iy, ix, 1]),
                depth=float(depth[b, iy, ix]) if depth is not None else None,
                keypoints=[None] * nk, keypoint_scores=[None] * nk, keypoint_affinities=[None] * nk))
        for k in range(keypoint_n_detections):
            ks = float(kscore[b, k])
            if ks < keypoint_score_threshold:
                break
            kl = int(klabel[b, k])
            owner, slot = keypoint_owner[kl]
            cands = [d for d in dets if d["label"] == owner and d["keypoints"][slot] is None]
            if not cands:
                continue
            kyi, kxi = kindex[b, k, 0], kindex[b, k, 1]
            ky = float(kyi / out_h)
            kx = float(kxi / out_w)
            ay = float(prediction.keypoint_affinity[b, kl, 0, kyi, kxi])
            ax = float(prediction.keypoint_affinity[b, kl, 1, kyi, kxi])
            ang = atan2(ay, ax)
            errs = [abs(ang - atan2(ky - d["y"], kx - d["x"])) for d in cands]
            best = cands[errs.index(min(errs))]
            best["keypoints"][slot] = (ky, kx)
            best["keypoint_affinities"][slot] = (ay, ax)
            best["keypoint_scores"][slot] = ks
        out.append(dets)
    return out
