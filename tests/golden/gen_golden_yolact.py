"""Generate YOLACT goldens.

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER: it imports the reference modules
src/tauv_vision/yolact/model/{config,anchors,boxes,nms,masks,masknet}.py read-only (they need
only torch). The .npz holds seeded inputs and the reference's outputs; no reference source.

Post-processing geometries: the reference's 640x360 training config (train.py:24-45: anchor
scales 24..384, aspect ratio 1, variances (0.1, 0.2), 7 classes, 8 prototypes; FPN levels
45x80 .. 3x5 -> 4835 anchors), BASELINE's 550x550 (69x69 .. 5x5 -> 6416 anchors), a 256x256
case with three aspect ratios, the reference's evaluate.py:17-34 config (640x360, aspect ratios
(1/2, 1, 2) -> 14505 anchors, 3 classes, 32 prototypes) with top_k up to a full sort, and a
degenerate-box case (zero-area boxes: 0/0 IoUs that torch.max propagates as NaN). Prototype
maps are smaller than the network's (the mask kernel is size-independent) to keep the fixtures
small; masks are stored for the first 24 detections.

Protonet (Masknet, masknet.py:8-55): tests/golden/recipe.py PROTONET_CASES — seeded weights in
the reference key layout and seeded fpn[0] inputs; full outputs for the small cases, a seeded
output sample + per-channel sums for the production-size ones.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_yolact.py [case ...]
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
sys.path.insert(0, HERE)
from recipe import PROTONET_CASES, protonet_inputs, protonet_sample_index  # noqa: E402

NMS_KEYS = ((100, 0.5, 0.05), (200, 0.3, 0.2), (50, 0.7, 0.0))
CASES = {
    "yolact_640x360": dict(in_w=640, in_h=360, fpn=[(45, 80), (23, 40), (12, 20), (6, 10), (3, 5)],
                           ars=(1,), n_classes=7, k=8, proto=(60, 96), seed=300),
    "yolact_550x550": dict(in_w=550, in_h=550, fpn=[(69, 69), (35, 35), (18, 18), (9, 9), (5, 5)],
                           ars=(1,), n_classes=7, k=8, proto=(46, 46), seed=301),
    # three aspect ratios (anchor blocks per ratio, anchors.py:23-37)
    "yolact_256x256_ar3": dict(in_w=256, in_h=256, fpn=[(32, 32), (16, 16), (8, 8), (4, 4), (2, 2)],
                               ars=(1, 0.5, 2), n_classes=3, k=4, proto=(64, 64), seed=302),
    # evaluate.py:17-34: 14505 anchors; top_k 2000 / 20000 exercise the multi-workgroup sort and
    # the full-length IoU pass (top_k > anchors keeps every anchor)
    "yolact_640x360_ar3": dict(in_w=640, in_h=360, fpn=[(45, 80), (23, 40), (12, 20), (6, 10), (3, 5)],
                               ars=(1 / 2, 1, 2), n_classes=3, k=32, proto=(45, 80), seed=303, batch=1,
                               nms_keys=NMS_KEYS + ((2000, 0.5, 0.05), (20000, 0.4, 0.3)), encode=True, slim=True),
}


def ref_config(ModelConfig, c):
    fields = {f: None for f in ModelConfig.__dataclass_fields__}
    fields.update(in_w=c["in_w"], in_h=c["in_h"], anchor_scales=(24, 48, 96, 192, 384),
                  anchor_aspect_ratios=c["ars"], box_variances=(0.1, 0.2))
    return ModelConfig(**fields)


def gen_postprocess(name, c, mods):
    ModelConfig, get_anchor, box_decode, box_encode, nms, assemble_mask = mods
    cfg = ref_config(ModelConfig, c)
    anchor = torch.cat([get_anchor(i, s, cfg) for i, s in enumerate(c["fpn"])], dim=1)
    A = anchor.shape[1]
    B = c.get("batch", 2)
    g = torch.Generator().manual_seed(c["seed"])
    enc = torch.randn(B, A, 4, generator=g) * 0.5
    box = box_decode(enc, anchor, cfg)
    cls = torch.randn(B, A, c["n_classes"] + 1, generator=g) * 2.0
    out = dict(anchor=anchor.numpy(), enc=enc.numpy(), box=box.numpy(), cls=cls.numpy(), A=np.array(A))
    for top_k, iou, conf in c.get("nms_keys", NMS_KEYS):
        det = nms(cls, box, top_k, iou, conf)
        out[f"nms_{top_k}_{iou}_{conf}"] = det.numpy()
    det = nms(cls, box, 100, 0.5, 0.05)
    proto = torch.randn(c["k"], *c["proto"], generator=g)
    coeff = torch.randn(B, A, c["k"], generator=g)
    out.update(proto=proto.numpy(), mask_det=det.numpy())
    if c.get("slim"):  # only the coefficient rows the masks use
        out.update(coeff_box=coeff[0, det[:24]].numpy(), coeff_nobox=coeff[0, det[:5]].numpy())
    else:
        out["coeff"] = coeff.numpy()
    out["mask_box"] = assemble_mask(proto, coeff[0, det[:24]], box[0, det[:24]]).numpy()
    out["mask_nobox"] = assemble_mask(proto, coeff[0, det[:5]], None).numpy()
    if c.get("encode"):
        # ground-truth-like boxes (y, x in [0, 1], h, w in [0.01, 0.5]) -> encodings (boxes.py:45-53)
        gt = torch.cat([torch.rand(B, A, 2, generator=g), torch.rand(B, A, 2, generator=g) * 0.49 + 0.01], -1)
        out["gt_box"] = gt.numpy()
        out["gt_enc"] = box_encode(gt.clone(), anchor, cfg).numpy()
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, "anchors", A, "kept", len(det), "mask", out["mask_box"].shape)


def gen_degenerate(mods):
    """Zero-area boxes (nms.py:19-24 over boxes.py:64-85): pairs of h = 0 / w = 0 boxes give 0/0
    IoUs; torch.max over the triu matrix returns NaN for such a column and NaN <= thr is False."""
    _, _, _, _, nms, _ = mods
    g = torch.Generator().manual_seed(320)
    A = 64
    box = torch.rand(1, A, 4, generator=g) * 0.4 + 0.05
    box[0, 0:8, 2] = 0.0    # h = 0
    box[0, 8:12, 3] = 0.0   # w = 0
    box[0, 12:16, 2:] = 0.0  # both
    box[0, 4:8, :2] = box[0, 0:4, :2]  # identical zero-area pairs
    cls = torch.randn(1, A, 4, generator=g) * 2.0
    out = dict(box=box.numpy(), cls=cls.numpy())
    for top_k, iou, conf in NMS_KEYS:
        out[f"nms_{top_k}_{iou}_{conf}"] = nms(cls, box, top_k, iou, conf).numpy()
    np.savez_compressed(os.path.join(HERE, "yolact_degenerate.npz"), **out)
    print("yolact_degenerate", {k: len(v) for k, v in out.items() if k.startswith("nms")})


def gen_protonet(case, Masknet, ModelConfig):
    fields = {f: None for f in ModelConfig.__dataclass_fields__}
    fields.update(feature_depth=case["F"], n_prototype_masks=case["k"])
    net = Masknet(ModelConfig(**fields)).eval()
    sd, x = protonet_inputs(case)
    net.load_state_dict(sd)
    with torch.no_grad():
        y = net(x)
    out = {"out_shape": np.array(y.shape), "chan_sum": y.double().sum(dim=(0, 2, 3)).numpy()}
    if case["full"]:
        out.update(x=x.numpy(), out=y.numpy())
    else:
        idx = protonet_sample_index(case)
        out.update(sample_index=idx.numpy(), sample=y.reshape(-1)[idx].numpy())
    np.savez_compressed(os.path.join(HERE, case["name"] + ".npz"), **out)
    print(case["name"], tuple(y.shape), "range", float(y.min()), float(y.max()))


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    from tauv_vision.yolact.model.config import ModelConfig
    from tauv_vision.yolact.model.anchors import get_anchor
    from tauv_vision.yolact.model.boxes import box_decode, box_encode
    from tauv_vision.yolact.model.nms import nms
    from tauv_vision.yolact.model.masks import assemble_mask
    from tauv_vision.yolact.model.masknet import Masknet
    want = set(sys.argv[1:])
    mods = (ModelConfig, get_anchor, box_decode, box_encode, nms, assemble_mask)
    for name, c in CASES.items():
        if not want or name in want:
            gen_postprocess(name, c, mods)
    if not want or "yolact_degenerate" in want:
        gen_degenerate(mods)
    for case in PROTONET_CASES:
        if not want or case["name"] in want:
            gen_protonet(case, Masknet, ModelConfig)


if __name__ == "__main__":
    main()
