"""Golden fixtures for the training-target generators (loss.py:31-135).

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER: it imports the reference's loss.py from
/root/reference/src (with inert stand-ins for the modules that file's imports pull in but
that generate_heatmap / generate_keypoint_heatmap / out_index_for_position never call:
cv2 and spatialmath via decode.py, torchvision.transforms.v2 via pose_dataset.py's
PoseSample.load), builds seeded PoseSample batches, and stores inputs + the reference's
outputs as tests/golden/targets_*.npz. Data only: the reference source does not travel.
    python tests/golden/gen_golden_targets.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def _import_reference():
    sys.dont_write_bytecode = True
    cv2 = types.ModuleType("cv2")
    sm = types.ModuleType("spatialmath")
    sm.SE3 = object
    sm.SO3 = object
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tvt2 = types.ModuleType("torchvision.transforms.v2")
    tv.transforms = tvt
    tvt.v2 = tvt2
    for name, mod in (("cv2", cv2), ("spatialmath", sm), ("torchvision", tv), ("torchvision.transforms", tvt),
                      ("torchvision.transforms.v2", tvt2)):
        sys.modules.setdefault(name, mod)
    sys.path.insert(0, REF_SRC)
    from tauv_vision.centernet.model import config as rcfg
    from tauv_vision.centernet.model import loss as rloss
    from tauv_vision.datasets.load import pose_dataset as rpose
    return rcfg, rloss, rpose


# (name, B, n_objects, n_labels, n_instances, n_keypoints, in_h, in_w, downsamples, kp sigma, aff sigma, seed)
CASES = [
    ("targets_b2_o5_l3_240x320", 2, 5, 3, 7, 4, 240, 320, 2, 2.0, 4.0, 11),
    ("targets_b3_o9_l4_480x640", 3, 9, 4, 12, 6, 480, 640, 2, 3.5, 6.0, 12),
    ("targets_b2_o4_l2_96x128_tinysigma", 2, 4, 2, 6, 3, 96, 128, 1, 0.05, 0.5, 13),
]


def make_case(rpose, B, n_obj, n_lab, n_inst, n_kp, seed, out_h, out_w):
    g = torch.Generator().manual_seed(seed)
    valid = torch.rand((B, n_obj), generator=g) < 0.8
    label = torch.randint(0, n_lab, (B, n_obj), generator=g)
    center = torch.rand((B, n_obj, 2), generator=g) * 1.1 - 0.05  # some centers off the frame
    # an object exactly on a cell center: the affinity's 0/0 at that cell (nan_to_num -> 0)
    center[0, 0] = torch.tensor([10.0 / out_h, 12.0 / out_w])
    size = torch.rand((B, n_obj, 2), generator=g) * 0.3
    kvalid = torch.rand((B, n_inst), generator=g) < 0.85
    klabel = torch.randint(0, n_kp, (B, n_inst), generator=g)
    kcenter = torch.rand((B, n_inst, 2), generator=g)
    kobj = torch.randint(0, n_obj, (B, n_inst), generator=g)
    # two instances of the same keypoint owned by the same object: equal distances (a tie: the
    # earlier instance keeps the cell)
    klabel[0, 1] = klabel[0, 0]
    kobj[0, 1] = kobj[0, 0]
    kvalid[0, :2] = True
    truth = rpose.PoseSample(img=torch.zeros((B, 3, 1, 1)), valid=valid, label=label, center=center, size=size,
                             roll=None, pitch=None, yaw=None, depth=None, keypoint_valid=kvalid,
                             keypoint_label=klabel, keypoint_center=kcenter, keypoint_object_index=kobj)
    return truth


def main():
    rcfg, rloss, rpose = _import_reference()
    for name, B, n_obj, n_lab, n_inst, n_kp, in_h, in_w, ds, ks, as_, seed in CASES:
        mc = rcfg.ModelConfig([2] * 5, [16] * 6, in_h, in_w, ds, 1.0)
        tc = rcfg.TrainConfig(lr=1e-3, batch_size=B, n_batches=1, n_epochs=1, heatmap_focal_loss_a=2.0,
                              heatmap_focal_loss_b=4.0, heatmap_sigma_factor=0.05, keypoint_heatmap_sigma=ks,
                              keypoint_affinity_sigma=as_, loss_lambda_keypoint_heatmap=1.0,
                              loss_lambda_keypoint_affinity=1.0, loss_lambda_size=1.0, loss_lambda_offset=1.0,
                              loss_lambda_angle=1.0, loss_lambda_depth=1.0, n_workers=0, weight_save_interval=1)
        oc = types.SimpleNamespace(n_labels=n_lab, n_keypoints=n_kp)
        truth = make_case(rpose, B, n_obj, n_lab, n_inst, n_kp, seed, mc.out_h, mc.out_w)
        heat = rloss.generate_heatmap(truth, mc, tc, oc)
        kh, kaw, kaff = rloss.generate_keypoint_heatmap(truth, mc, tc, oc)
        idx = rloss.out_index_for_position(truth.center, mc)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"),
            in_h=in_h, in_w=in_w, downsamples=ds, n_labels=n_lab, n_keypoints=n_kp,
            keypoint_heatmap_sigma=ks, keypoint_affinity_sigma=as_,
            valid=truth.valid.numpy(), label=truth.label.numpy(), center=truth.center.numpy(),
            keypoint_valid=truth.keypoint_valid.numpy(), keypoint_label=truth.keypoint_label.numpy(),
            keypoint_center=truth.keypoint_center.numpy(), keypoint_object_index=truth.keypoint_object_index.numpy(),
            heatmap=heat.numpy(), keypoint_heatmap=kh.numpy(), keypoint_affinity_weight=kaw.numpy(),
            keypoint_affinity=kaff.numpy(), out_index=idx.numpy())
        print(name, tuple(heat.shape), tuple(kaff.shape), float(heat.max()), float(kaff.abs().max()))


if __name__ == "__main__":
    main()
