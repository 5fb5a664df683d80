"""Generate YOLACT post-processing goldens.

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER: it imports the reference modules
src/tauv_vision/yolact/model/{config,anchors,boxes,nms,masks}.py read-only (they need only
torch). The .npz holds seeded inputs and the reference's outputs; no reference source.
Geometries: the reference's 640x360 training config (train.py:24-45: anchor scales
24..384, aspect ratio 1, variances (0.1, 0.2), 7 classes, 8 prototypes; FPN levels 45x80 ..
3x5 -> 4835 anchors), BASELINE's 550x550 (69x69 .. 5x5 -> 6416 anchors) and a 256x256 case
with three aspect ratios. Prototype maps are smaller than the network's (the mask kernel is
size-independent) to keep the fixtures small; masks are stored for the first 24 detections.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_yolact.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"

CASES = {
    "yolact_640x360": dict(in_w=640, in_h=360, fpn=[(45, 80), (23, 40), (12, 20), (6, 10), (3, 5)],
                           ars=(1,), n_classes=7, k=8, proto=(60, 96), seed=300),
    "yolact_550x550": dict(in_w=550, in_h=550, fpn=[(69, 69), (35, 35), (18, 18), (9, 9), (5, 5)],
                           ars=(1,), n_classes=7, k=8, proto=(46, 46), seed=301),
    # three aspect ratios (anchor blocks per ratio, anchors.py:23-37)
    "yolact_256x256_ar3": dict(in_w=256, in_h=256, fpn=[(32, 32), (16, 16), (8, 8), (4, 4), (2, 2)],
                               ars=(1, 0.5, 2), n_classes=3, k=4, proto=(64, 64), seed=302),
}


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    from tauv_vision.yolact.model.config import ModelConfig
    from tauv_vision.yolact.model.anchors import get_anchor
    from tauv_vision.yolact.model.boxes import box_decode
    from tauv_vision.yolact.model.nms import nms
    from tauv_vision.yolact.model.masks import assemble_mask
    for name, c in CASES.items():
        fields = {f: None for f in ModelConfig.__dataclass_fields__}
        fields.update(in_w=c["in_w"], in_h=c["in_h"], anchor_scales=(24, 48, 96, 192, 384),
                      anchor_aspect_ratios=c["ars"], box_variances=(0.1, 0.2))
        cfg = ModelConfig(**fields)
        anchor = torch.cat([get_anchor(i, s, cfg) for i, s in enumerate(c["fpn"])], dim=1)
        A = anchor.shape[1]
        g = torch.Generator().manual_seed(c["seed"])
        enc = torch.randn(2, A, 4, generator=g) * 0.5
        box = box_decode(enc, anchor, cfg)
        cls = torch.randn(2, A, c["n_classes"] + 1, generator=g) * 2.0
        out = dict(anchor=anchor.numpy(), enc=enc.numpy(), box=box.numpy(), cls=cls.numpy(), A=np.array(A))
        for top_k, iou, conf in ((100, 0.5, 0.05), (200, 0.3, 0.2), (50, 0.7, 0.0)):
            det = nms(cls, box, top_k, iou, conf)
            out[f"nms_{top_k}_{iou}_{conf}"] = det.numpy()
        det = nms(cls, box, 100, 0.5, 0.05)
        proto = torch.randn(c["k"], *c["proto"], generator=g)
        coeff = torch.randn(2, A, c["k"], generator=g)
        out.update(proto=proto.numpy(), coeff=coeff.numpy(), mask_det=det.numpy())
        out["mask_box"] = assemble_mask(proto, coeff[0, det[:24]], box[0, det[:24]]).numpy()
        out["mask_nobox"] = assemble_mask(proto, coeff[0, det[:5]], None).numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, "anchors", A, "kept", len(det), "mask", out["mask_box"].shape)


if __name__ == "__main__":
    main()
