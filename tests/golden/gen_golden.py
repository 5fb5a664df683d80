"""Generate the golden vectors that pin the oracle (and, through it, the HIP path).

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER: it imports the reference
(Tartan-AUV/TAUV-Vision @ 2024_10_08) from /root/reference/src, read-only, with
inert stand-ins for the two modules its decode file imports but never calls on
these paths (`cv2`, used only by `decode_keypoints` once >= 6 keypoints match,
decode.py:141-172; `spatialmath`, type annotations only, decode.py:10,48).
Nothing produced here contains reference source: the .npz files hold inputs and
outputs only (plus the state_dict key list / shapes, which is the weight-file
format the drop-in must accept).

Weights are NOT committed. They come from the seeded recipe in
`tests/golden/recipe.py` (shared with the tests, which regenerate them and
check a per-key checksum against the one stored here).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from recipe import (MODEL_CASES, seeded_state_dict, seeded_input,  # noqa: E402
                    decode_case_inputs, gaussian_blob, squares_batch)

REF_SRC = "/root/reference/src"


def _import_reference():
    sys.dont_write_bytecode = True
    cv2 = types.ModuleType("cv2")
    sm = types.ModuleType("spatialmath")
    sm.SE3 = object
    sm.SO3 = object
    sys.modules.setdefault("cv2", cv2)
    sys.modules.setdefault("spatialmath", sm)
    sys.path.insert(0, REF_SRC)
    from tauv_vision.centernet.model import config as rcfg
    from tauv_vision.centernet.model import centernet as rnet
    from tauv_vision.centernet.model import decode as rdec
    from tauv_vision.centernet.model.backbones import dla as rdla
    return rcfg, rnet, rdec, rdla


def object_config_for(rcfg, spec):
    """spec: dict(n_labels, keypoints_per_label, depth, yaw, pitch, roll)."""
    configs = []
    for i in range(spec["n_labels"]):
        kps = spec.get("keypoints_per_label", 0)
        configs.append(rcfg.ObjectConfig(
            id=f"obj{i}",
            yaw=rcfg.AngleConfig(train=spec.get("yaw", False), modulo=2 * np.pi),
            pitch=rcfg.AngleConfig(train=spec.get("pitch", False), modulo=2 * np.pi),
            roll=rcfg.AngleConfig(train=spec.get("roll", False), modulo=2 * np.pi),
            train_depth=spec.get("depth", False),
            train_keypoints=kps > 0,
            keypoints=[(0.0, 0.0, 0.0)] * kps if kps > 0 else None,
        ))
    return rcfg.ObjectConfigSet(configs=configs)


def gen_models(rcfg, rnet, rdla, rdec):
    index = {}
    for case in MODEL_CASES:
        name = case["name"]
        torch.manual_seed(0)
        oc = object_config_for(rcfg, case["objects"])
        backbone = rdla.DLABackbone(case["heights"], case["channels"], case["downsamples"])
        model = rnet.Centernet(backbone, oc).eval()
        ref_sd = model.state_dict()
        keys = [(k, list(v.shape)) for k, v in ref_sd.items()]
        sd = seeded_state_dict(keys)
        model.load_state_dict(sd)
        img = seeded_input(case)
        with torch.no_grad():
            pred = model(img)
        out = {"img_checksum": np.array([float(img.double().sum()), float(img.double().abs().sum())])}
        fields = ["heatmap", "keypoint_heatmap", "keypoint_affinity", "size", "offset",
                  "roll_bin", "roll_offset", "pitch_bin", "pitch_offset", "yaw_bin",
                  "yaw_offset", "depth"]
        present = []
        for f in fields:
            t = getattr(pred, f)
            if t is not None:
                out[f] = t.contiguous().numpy()
                present.append(f)
        head_channels = rnet.get_head_channels(oc)
        mc = rcfg.ModelConfig(backbone_heights=case["heights"], backbone_channels=case["channels"],
                              in_h=case["in_h"], in_w=case["in_w"], downsamples=case["downsamples"],
                              angle_bin_overlap=float(np.pi / 3))
        # decode() on the network output (box path; depth where present)
        for thr in (0.05, 0.3):
            dets = rdec.decode(pred, mc, 20, thr)
            out[f"decode_thr{thr}"] = _pack_dets(dets, 20, has_depth=pred.depth is not None)
        # the bench's decode (K=100) with no threshold cut: every top-100 peak's record, so the
        # fp16/bf16 paths' peak-set agreement and box error are measured against the reference
        out["decode_k100"] = _pack_dets(rdec.decode(pred, mc, 100, 0.0), 100, has_depth=pred.depth is not None)
        out["decode_k100_index"] = _flat_peaks(rdec, pred.heatmap, 100)
        if oc.train_keypoints:
            kd = rdec.decode_keypoints(pred, mc, oc, np.eye(3), n_detections=10, keypoint_n_detections=50,
                                       score_threshold=0.05, keypoint_score_threshold=0.05,
                                       keypoint_angle_threshold=0.3)
            out["decode_keypoints"] = _pack_kp_dets(kd, 10, oc)
        checks = np.array([[float(v.double().sum()), float(v.double().abs().sum())]
                           if v.dtype.is_floating_point else [float(v), 0.0] for _, v in sd.items()])
        out["weight_checksums"] = checks
        np.savez_compressed(os.path.join(HERE, f"model_{name}.npz"), **out)
        index[name] = {"keys": keys, "head_channels": head_channels, "fields": present,
                       "case": case, "n_params": int(sum(int(np.prod(s)) for _, s in keys))}
        print(f"{name}: {len(keys)} keys, heads {head_channels}, heatmap {tuple(pred.heatmap.shape)}")
    with open(os.path.join(HERE, "models.json"), "w") as f:
        json.dump(index, f, indent=1)


def _pack_dets(dets, K, has_depth):
    """[B, K, 8]: label, score, y, x, h, w, depth, valid; NaN-padded."""
    B = len(dets)
    rec = np.full((B, K, 8), np.nan, dtype=np.float64)
    for b, ds in enumerate(dets):
        for i, d in enumerate(ds):
            rec[b, i, :6] = [float(d.label), float(d.score), d.y, d.x, d.h, d.w]
            rec[b, i, 6] = d.depth if (has_depth and d.depth is not None) else np.nan
            rec[b, i, 7] = 1.0
    return rec


def _flat_peaks(rdec, heatmap, K):
    """[B, K] int64 flat peak indices (label*H*W + y*W + x) of the reference's own
    sigmoid -> heatmap_nms -> heatmap_detect chain (decode.py:182-184), in its order."""
    import torch.nn.functional as F
    H, W = heatmap.shape[2:]
    idx, lab, _ = rdec.heatmap_detect(rdec.heatmap_nms(F.sigmoid(heatmap), 3), K)
    return (lab * H * W + idx[..., 0] * W + idx[..., 1]).numpy()


def _pack_kp_dets(dets, K, oc):
    """[B, K, 7 + 5*max_kp]: label, score, y, x, h, w, valid, then per keypoint
    (ky, kx, score, aff_y, aff_x); NaN where absent."""
    max_kp = max(len(c.keypoints) for c in oc.configs if c.keypoints is not None)
    B = len(dets)
    rec = np.full((B, K, 7 + 5 * max_kp), np.nan, dtype=np.float64)
    for b, ds in enumerate(dets):
        for i, d in enumerate(ds):
            rec[b, i, :7] = [d.label, d.score, d.y, d.x, d.h, d.w, 1.0]
            for j, kp in enumerate(d.keypoints):
                if kp is not None:
                    rec[b, i, 7 + 5 * j: 12 + 5 * j] = [kp[0], kp[1], d.keypoint_scores[j],
                                                        d.keypoint_affinities[j][0], d.keypoint_affinities[j][1]]
    return rec


def _tie_free_seed(B, C, H, W, seed, K):
    """First seed >= `seed` whose sigmoid map has no equal 3x3 neighbours and a strictly
    ordered top-(K+1) after NMS, so peak sets and top-K order are fully determined."""
    for s in range(seed, seed + 10000, 1000):
        logits = decode_case_inputs(B, C, H, W, s)[0]
        sig = torch.sigmoid(logits)
        pad = torch.nn.functional.pad(sig, (1, 1, 1, 1), value=-1.0)
        ties = False
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if dy == 0 and dx == 0:
                    continue
                nb = pad[:, :, 1 + dy:1 + dy + H, 1 + dx:1 + dx + W]
                ties |= bool((nb == sig).any())
        peaks = (torch.nn.functional.max_pool2d(sig, 3, 1, 1) == sig).float() * sig
        top = torch.sort(peaks.reshape(B, -1), dim=1, descending=True).values[:, :K + 1]
        if not ties and bool((top[:, :-1] > top[:, 1:]).all()):
            return s
    raise RuntimeError("no tie-free seed")


def gen_decode(rnet, rdec, rcfg):
    """Decode-level goldens on seeded tie-free logits."""
    for name, (B, C, H, W, in_h, in_w, ds, seed) in {
        "decode_b3_c4_120x160": (3, 4, 120, 160, 480, 640, 2, 11),
        "decode_b2_c4_90x160": (2, 4, 90, 160, 360, 640, 2, 12),
        "decode_b1_c80_64x64": (1, 80, 64, 64, 256, 256, 2, 13),
    }.items():
        seed = _tie_free_seed(B, C, H, W, seed, 100)
        logits, size, offset, depth = decode_case_inputs(B, C, H, W, seed)
        mc = rcfg.ModelConfig(backbone_heights=[], backbone_channels=[], in_h=in_h, in_w=in_w,
                              downsamples=ds, angle_bin_overlap=1.0)
        sig = torch.sigmoid(logits)
        nms = rdec.heatmap_nms(sig, kernel_size=3)
        K = 100
        idx, lab, score = rdec.heatmap_detect(nms, K)
        # tie-freeness of what the tests compare (torch.topk tie order is unspecified)
        s_sorted = torch.sort(nms.reshape(B, -1), dim=1, descending=True).values
        assert bool((s_sorted[:, :K] > s_sorted[:, 1:K + 1]).all()), "ties in top-K: reseed"
        pred = rnet.Prediction(heatmap=logits, keypoint_heatmap=None, keypoint_affinity=None,
                               size=size, offset=offset, roll_bin=None, roll_offset=None,
                               pitch_bin=None, pitch_offset=None, yaw_bin=None, yaw_offset=None,
                               depth=depth)
        out = dict(seed=np.array([seed, B, C, H, W]), nms=nms.numpy(), index=idx.numpy(), label=lab.numpy(),
                   score=score.numpy(), meta=np.array([in_h, in_w, ds]),
                   input_checksums=np.array([float(t.double().sum()) for t in (logits, size, offset, depth)]))
        for thr in (0.05, 0.3, 0.9):
            out[f"decode_thr{thr}"] = _pack_dets(rdec.decode(pred, mc, K, thr), K, has_depth=True)
        pred.depth = None
        out["decode_nodepth_thr0.3"] = _pack_dets(rdec.decode(pred, mc, K, 0.3), K, has_depth=False)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, "ok")


def gen_kat(rdec):
    """decode.py:327-339 self-check, restated with the loss.py:64-67 Gaussian form."""
    h = torch.cat((gaussian_blob(512, 512, 100, 100, 50).unsqueeze(0).unsqueeze(1),
                   gaussian_blob(512, 512, 200, 200, 50).unsqueeze(0).unsqueeze(1)), dim=1)
    nms = rdec.heatmap_nms(h, 3)
    idx, lab, score = rdec.heatmap_detect(nms, 100)
    np.savez_compressed(os.path.join(HERE, "kat_two_blobs.npz"), index=idx[:, :2].numpy(),
                        label=lab[:, :2].numpy(), score=score[:, :2].numpy())
    print("kat", idx[0, :3].tolist(), lab[0, :3].tolist(), score[0, :3].tolist())


def gen_pad_to_match(rdla):
    """dla.py:195-209 incl. the (above,below,left,right) -> (W_l,W_r,H_t,H_b) quirk."""
    g = torch.Generator().manual_seed(5)
    cases = [((16, 20), (15, 20)), ((128, 160), (120, 160)), ((96, 160), (90, 160)),
             ((92, 160), (90, 160)), ((24, 40), (23, 40)), ((8, 10), (8, 10)), ((32, 32), (24, 32)),
             ((6, 12), (6, 9)), ((10, 8), (7, 8))]
    out = {}
    for i, (fs, ts) in enumerate(cases):
        f = torch.randn((1, 2) + fs, generator=g)
        r = rdla.pad_to_match(f, torch.Size((1, 2) + ts))
        out[f"in{i}"] = f.numpy()
        out[f"out{i}"] = r.contiguous().numpy()
        out[f"shape{i}"] = np.array(ts)
    np.savez_compressed(os.path.join(HERE, "pad_to_match.npz"), **out)
    print("pad_to_match ok")


def gen_squares():
    """Synthetic rotated-square frames (tests/centernet_square_detection.py:64-126, no cv2)."""
    img, centers = squares_batch(4, 128, 128, seed=3)
    np.savez_compressed(os.path.join(HERE, "squares_b4_128.npz"), img=img.numpy(), centers=centers)


if __name__ == "__main__":
    rcfg, rnet, rdec, rdla = _import_reference()
    gen_kat(rdec)
    gen_pad_to_match(rdla)
    gen_decode(rnet, rdec, rcfg)
    gen_squares()
    gen_models(rcfg, rnet, rdla, rdec)
