"""Seeded, documented recipes shared by the golden generator and the tests.

Everything here is plain torch/numpy written for this repo (no reference code):
model cases, the seeded weight recipe (with small random conv
biases so bias paths are exercised), seeded inputs, tie-free decode inputs, the
Gaussian blob of the decode.py:327-339 known-answer test (loss.py:64-67 form) and
a cv2-free restatement of the synthetic rotated-square frames of
tests/centernet_square_detection.py:64-126.
"""
import math

import numpy as np
import torch

PLAIN4 = {"n_labels": 4}

MODEL_CASES = [
    # "R18" map at reduced width/size; the pad_to_match column shift fires (32->24 rows).
    dict(name="r18_c16_b2_96x128", heights=[2] * 5, channels=[16] * 6, downsamples=2,
         in_h=96, in_w=128, batch=2, seed=100, objects=PLAIN4),
    # every optional head (yaw/pitch/roll bins+offsets, depth): exercises the head pop order
    # quirk (get_head_channels yaw,pitch,roll vs forward roll,pitch,yaw; centernet.py:77-90,133-140).
    dict(name="r18_c32_b1_96x128_allheads", heights=[2] * 5, channels=[32] * 6, downsamples=2,
         in_h=96, in_w=128, batch=1, seed=101,
         objects={"n_labels": 2, "yaw": True, "pitch": True, "roll": True, "depth": True}),
    # samples_torpedo.py:4-82 geometry (360x640, 4 labels x 1 keypoint), reduced width.
    dict(name="torpedo_c16_b1_360x640", heights=[2] * 5, channels=[16] * 6, downsamples=2,
         in_h=360, in_w=640, batch=1, seed=102, objects={"n_labels": 4, "keypoints_per_label": 1}),
    # tests/centernet_square_detection.py:21-61 intent: [2]*6 / [32]*7, ratio 2, one yaw class.
    dict(name="square_c32_b2_128", heights=[2] * 6, channels=[32] * 7, downsamples=1,
         in_h=128, in_w=128, batch=2, seed=103, objects={"n_labels": 1, "yaw": True}, squares=True),
    # height-1 trees and per-level channel widths (dla.py:419-429 shape family).
    dict(name="dla_var_b1_128x128", heights=[1, 2, 2, 1], channels=[16, 16, 32, 32, 64], downsamples=1,
         in_h=128, in_w=128, batch=1, seed=104, objects=PLAIN4),
    # the production-width "R18" at the BASELINE resolution.
    dict(name="r18_c128_b1_480x640", heights=[2] * 5, channels=[128] * 6, downsamples=2,
         in_h=480, in_w=640, batch=1, seed=105, objects=PLAIN4),
]

# CenterpointDLA34 (centerpoint_dla.py:544-578; DLA-34 levels/channels fixed by dla34(),
# :309-315) — SURVEY §8a a12-a15.
DLA34_CASES = [
    # small frames, batch 2, the plain 4-class heads [4, 2, 2]
    dict(name="b2_64x96", in_h=64, in_w=96, batch=2, seed=200, objects=PLAIN4),
    # 120x96: ceil-mode max-pool (15 -> 8 rows), pad_to_match crops (16 -> 15) and, in ida_up
    # (f = 4: 32 -> 30 rows), the one-row downward shift; keypoint heads [4, 4, 8, 2, 2]
    dict(name="b1_120x96_kp", in_h=120, in_w=96, batch=1, seed=201,
         objects={"n_labels": 4, "keypoints_per_label": 1}),
    # the BASELINE geometry (480x640) with the north-star DLA34 heads [4, 4, 8, 2, 2]
    dict(name="b1_480x640_kp", in_h=480, in_w=640, batch=1, seed=202,
         objects={"n_labels": 4, "keypoints_per_label": 1}),
    # the production node's configuration (centernet_node.py:46 with samples_torpedo.py:4-82):
    # 360x640, 4 labels x 1 keypoint; ida_up's pad_to_match shifts one row (92 -> 90, a14)
    dict(name="b1_360x640_kp", in_h=360, in_w=640, batch=1, seed=203,
         objects={"n_labels": 4, "keypoints_per_label": 1}),
]

# YOLACT Masknet protonet (masknet.py:8-55): feature_depth F, n_prototype_masks k, fpn[0] size.
# Small cases store the full output; the production-size cases (train.py:28-33 config F=256, k=8
# at the 640x360 fpn[0] of 45x80 and BASELINE's 550x550 -> 69x69) store a seeded sample of output
# positions plus per-channel float64 sums, and the tests regenerate inputs / weights from the seeds.
PROTONET_CASES = [
    dict(name="protonet_f32_k8_b2_12x20", F=32, k=8, batch=2, H=12, W=20, seed=310, full=True),
    dict(name="protonet_f64_k16_b1_9x17", F=64, k=16, batch=1, H=9, W=17, seed=311, full=True),
    dict(name="protonet_f256_k8_b1_45x80", F=256, k=8, batch=1, H=45, W=80, seed=312, full=False),
    dict(name="protonet_f256_k8_b1_69x69", F=256, k=8, batch=1, H=69, W=69, seed=313, full=False),
]
PROTONET_SAMPLES = 4096


def protonet_case(name):
    for c in PROTONET_CASES:
        if c["name"] == name:
            return c
    raise KeyError(name)


def protonet_layout(F, k):
    """masknet.py:13-41 registration order (the reference Masknet.state_dict() keys)."""
    out = []
    for i, up in ((1, True), (2, True), (3, False)):
        out += [(f"_layers_{i}.0.0.weight", (F, F, 3, 3)), (f"_layers_{i}.0.0.bias", (F,))]
        if up:
            out += [(f"_upsample_layer_{i}.weight", (F, F, 3, 3)), (f"_upsample_layer_{i}.bias", (F,))]
    out += [("_output_layer.weight", (k, F, 1, 1)), ("_output_layer.bias", (k,))]
    return out


def protonet_inputs(case):
    """(state_dict, fpn[0] input [B, F, H, W]) of a protonet case."""
    sd = seeded_state_dict(protonet_layout(case["F"], case["k"]), conv_seed=case["seed"], aux_seed=case["seed"] + 1)
    g = torch.Generator().manual_seed(case["seed"] + 2)
    x = torch.randn((case["batch"], case["F"], case["H"], case["W"]), generator=g)
    return sd, x


def protonet_sample_index(case):
    """Seeded flat output positions of the sampled (full=False) cases."""
    B, k, Ho, Wo = case["batch"], case["k"], 4 * case["H"], 4 * case["W"]
    g = torch.Generator().manual_seed(case["seed"] + 3)
    return torch.randint(0, B * k * Ho * Wo, (PROTONET_SAMPLES,), generator=g)


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def case_by_name(name):
    for c in MODEL_CASES:
        if c["name"] == name:
            return c
    raise KeyError(name)


def seeded_state_dict(keys_shapes, conv_seed=0, aux_seed=1):
    """Deterministic weights for a state_dict key list (order matters).

    conv / conv-transpose weights (4-D): xavier_uniform from generator(conv_seed)
    (bound = sqrt(6 / ((d0 + d1) * kh * kw)), torch's fan rule for both kinds).
    From generator(aux_seed), in key order: BN weight ~ U(0.75, 1.25), BN bias ~
    N(0, 0.1^2), running_mean ~ N(0, 0.1^2), running_var ~ U(0.75, 1.25); conv bias ~
    U(-0.1, 0.1). num_batches_tracked = 0.
    """
    g_conv = torch.Generator().manual_seed(conv_seed)
    g_aux = torch.Generator().manual_seed(aux_seed)
    names = {k for k, _ in keys_shapes}
    sd = {}
    for k, shape in keys_shapes:
        prefix, leaf = k.rsplit(".", 1)
        is_bn = (prefix + ".running_mean") in names
        shape = tuple(shape)
        if leaf == "num_batches_tracked":
            sd[k] = torch.tensor(0, dtype=torch.long)
        elif leaf == "running_mean":
            sd[k] = torch.randn(shape, generator=g_aux) * 0.1
        elif leaf == "running_var":
            sd[k] = torch.rand(shape, generator=g_aux) * 0.5 + 0.75
        elif len(shape) == 4:
            rf = shape[2] * shape[3]
            bound = math.sqrt(6.0 / ((shape[0] + shape[1]) * rf))
            sd[k] = (torch.rand(shape, generator=g_conv) * 2.0 - 1.0) * bound
        elif is_bn and leaf == "weight":
            sd[k] = torch.rand(shape, generator=g_aux) * 0.5 + 0.75
        elif is_bn and leaf == "bias":
            sd[k] = torch.randn(shape, generator=g_aux) * 0.1
        elif leaf == "bias":
            sd[k] = (torch.rand(shape, generator=g_aux) * 2.0 - 1.0) * 0.1
        else:
            raise ValueError(f"unexpected parameter {k} {shape}")
    return sd


def normalize(img01, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    m = torch.tensor(mean, dtype=torch.float32).view(1, 3, 1, 1)
    s = torch.tensor(std, dtype=torch.float32).view(1, 3, 1, 1)
    return (img01 - m) / s


def seeded_input(case):
    B, H, W = case["batch"], case["in_h"], case["in_w"]
    if case.get("squares"):
        img, _ = squares_batch(B, H, W, seed=case["seed"])
        return normalize(img, (0.51, 0.48, 0.48), (0.29, 0.29, 0.29))
    g = torch.Generator().manual_seed(case["seed"])
    u8 = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8)
    return normalize(u8.permute(0, 3, 1, 2).float() / 255.0)


def seeded_u8_frames(B, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8)


def decode_case_inputs(B, C, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    logits = torch.rand((B, C, H, W), generator=g) * 9.0 - 8.0
    size = torch.randn((B, H, W, 2), generator=g) * 10.0 + 20.0
    offset = torch.rand((B, H, W, 2), generator=g) * 4.0
    depth = torch.randn((B, H, W, 1), generator=g)
    return logits, size, offset, depth


def gaussian_blob(h, w, cy, cx, sigma):
    y = torch.arange(h, dtype=torch.float32).view(h, 1)
    x = torch.arange(w, dtype=torch.float32).view(1, w)
    return torch.exp(-((x - cx) ** 2 + (y - cy) ** 2) / (2 * sigma ** 2))


def _segment_dist(px, py, ax, ay, bx, by):
    vx, vy = bx - ax, by - ay
    t = ((px - ax) * vx + (py - ay) * vy) / max(vx * vx + vy * vy, 1e-9)
    t = np.clip(t, 0.0, 1.0)
    dx, dy = px - (ax + t * vx), py - (ay + t * vy)
    return np.sqrt(dx * dx + dy * dy)


def squares_batch(B, H, W, seed):
    """Uniform-noise RGB frames with a red rotated-square outline (thickness 0.2*size/2)."""
    rng = np.random.default_rng(seed)
    imgs = np.zeros((B, 3, H, W), dtype=np.float32)
    centers = np.zeros((B, 2), dtype=np.int64)
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    for b in range(B):
        side = float(rng.uniform(H / 10, H / 4))
        cy = int(rng.uniform(H / 4, 3 * H / 4))
        cx = int(rng.uniform(W / 4, 3 * W / 4))
        yaw = float(rng.uniform(0, math.pi / 2))
        thick = max(1.0, math.floor(0.2 * side))
        c, s = math.cos(yaw), math.sin(yaw)
        corners = [(-side / 2, -side / 2), (side / 2, -side / 2), (side / 2, side / 2), (-side / 2, side / 2)]
        pts = [(cx + c * px - s * py, cy + s * px + c * py) for px, py in corners]
        d = np.full((H, W), np.inf)
        for i in range(4):
            ax, ay = pts[i]
            bx, by = pts[(i + 1) % 4]
            d = np.minimum(d, _segment_dist(xx, yy, ax, ay, bx, by))
        img = (255 * rng.random((H, W, 3))).astype(np.uint8)
        mask = d <= thick / 2
        img[mask] = (255, 0, 0)
        imgs[b] = img.transpose(2, 0, 1).astype(np.float32) / 255.0
        centers[b] = (cy, cx)
    return torch.from_numpy(imgs), centers
