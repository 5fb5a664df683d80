"""Shared test helpers: golden fixtures, seeded weights, object-config flags."""
import json
import os

import numpy as np
import torch

from recipe import MODEL_CASES, case_by_name, seeded_state_dict, seeded_input  # noqa: F401

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_MODELS = None


def models_index():
    global _MODELS
    if _MODELS is None:
        with open(os.path.join(GOLDEN, "models.json")) as f:
            _MODELS = json.load(f)
    return _MODELS


_MEASURED = {}


def record_measurement(key, value):
    """Collect measured drift (env TV_PARITY_OUT = JSON path) so tolerances can be set from
    numbers measured on MI355X; profiles/r2/parity_lowp.json is such a file."""
    _MEASURED[key] = value
    out = os.environ.get("TV_PARITY_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(_MEASURED, f, indent=1, sort_keys=True)


def golden(name):
    return np.load(os.path.join(GOLDEN, name if name.endswith(".npz") else name + ".npz"))


def case_flags(case):
    o = case["objects"]
    return dict(keypoints=o.get("keypoints_per_label", 0) > 0, yaw=o.get("yaw", False),
                pitch=o.get("pitch", False), roll=o.get("roll", False), depth=o.get("depth", False))


def case_state_dict(name):
    """Seeded weights for a model case, checked against the checksums the reference run stored."""
    entry = models_index()[name]
    sd = seeded_state_dict([(k, s) for k, s in entry["keys"]])
    checks = golden(f"model_{name}")["weight_checksums"]
    got = np.array([[float(v.double().sum()), float(v.double().abs().sum())]
                    if v.dtype.is_floating_point else [float(v), 0.0] for v in sd.values()])
    # double sums of large tensors depend on the host's reduction threading: compare to 1e-10
    assert np.allclose(got, checks, rtol=1e-10, atol=1e-12), "seeded weight recipe drifted from the golden run"
    return sd


def case_input(name):
    case = case_by_name(name)
    img = seeded_input(case)
    chk = golden(f"model_{name}")["img_checksum"]
    got = [float(img.double().sum()), float(img.double().abs().sum())]
    assert np.allclose(got, chk, rtol=1e-10, atol=1e-9), "seeded input drifted from the golden run"
    return img


def keypoint_owner(case):
    o = case["objects"]
    owner = []
    for lab in range(o["n_labels"]):
        for slot in range(o.get("keypoints_per_label", 0)):
            owner.append((lab, slot))
    return owner


# ---- CenterpointDLA34 cases (tests/golden/gen_golden_dla34.py) ----
_DLA34 = None


def dla34_index():
    global _DLA34
    if _DLA34 is None:
        with open(os.path.join(GOLDEN, "models_dla34.json")) as f:
            _DLA34 = json.load(f)
    return _DLA34


def dla34_state_dict(name):
    """Seeded reference-layout weights (keys `model.*`), checked against the golden run's checksums."""
    entry = dla34_index()[name]
    sd = seeded_state_dict([(k, s) for k, s in entry["keys"]])
    checks = golden(f"dla34_{name}")["weight_checksums"]
    got = np.array([[float(v.double().sum()), float(v.double().abs().sum())]
                    if v.dtype.is_floating_point else [float(v), 0.0] for v in sd.values()])
    assert np.allclose(got, checks, rtol=1e-10, atol=1e-12), "seeded weight recipe drifted from the golden run"
    return sd


def dla34_input(name):
    case = dla34_index()[name]["case"]
    img = seeded_input(case)
    chk = golden(f"dla34_{name}")["img_checksum"]
    got = [float(img.double().sum()), float(img.double().abs().sum())]
    assert np.allclose(got, chk, rtol=1e-10, atol=1e-9), "seeded input drifted from the golden run"
    return img
