"""CPU oracle for the TAUV-Vision CenterNet hot path — TEST INFRASTRUCTURE ONLY.

This package restates the reference's algorithm (Tartan-AUV/TAUV-Vision @ 2024_10_08)
as plain PyTorch-CPU code, op for op in the reference's order, so that on CPU it is
bit-identical to the reference. It is pinned against golden vectors produced by
importing the reference itself in the build container (tests/golden/gen_golden.py;
checked by tests/test_oracle_golden.py).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import it, and only as the checker / the timed CPU baseline. The product path
(`tauv-vision_amd/`) never imports it and has no CPU fallback.
"""
from .ref_forward import centernet_forward, backbone_forward, pad_to_match, head_channels_for, PredictionRef  # noqa: F401
from .ref_decode import (heatmap_nms, heatmap_detect, decode, decode_keypoints,  # noqa: F401
                         depth_decode)
from .ref_preprocess import preprocess  # noqa: F401
