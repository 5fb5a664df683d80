"""Pin the CPU oracle against the golden vectors produced by the reference itself
(tests/golden/gen_golden.py). CPU only."""
import numpy as np
import pytest
import torch

import oracle
from helpers import golden, models_index, case_by_name, case_flags, case_state_dict, case_input, keypoint_owner
from recipe import decode_case_inputs, gaussian_blob

FIELDS = ["heatmap", "keypoint_heatmap", "keypoint_affinity", "size", "offset", "roll_bin",
          "roll_offset", "pitch_bin", "pitch_offset", "yaw_bin", "yaw_offset", "depth"]


def test_kat_two_blobs():
    """decode.py:327-339 self-check (restated Gaussian)."""
    h = torch.cat((gaussian_blob(512, 512, 100, 100, 50)[None, None],
                   gaussian_blob(512, 512, 200, 200, 50)[None, None]), dim=1)
    idx, lab, score = oracle.heatmap_detect(oracle.heatmap_nms(h, 3), 100)
    g = golden("kat_two_blobs")
    assert idx[0, 0].tolist() == [100, 100]
    np.testing.assert_array_equal(idx[:, :2].numpy(), g["index"])
    np.testing.assert_array_equal(lab[:, :2].numpy(), g["label"])
    np.testing.assert_array_equal(score[:, :2].numpy(), g["score"])


def test_pad_to_match_quirk():
    g = golden("pad_to_match")
    n = len([k for k in g.files if k.startswith("in")])
    for i in range(n):
        f = torch.from_numpy(g[f"in{i}"])
        shape = torch.Size(tuple(f.shape[:2]) + tuple(g[f"shape{i}"]))
        np.testing.assert_array_equal(oracle.pad_to_match(f, shape).contiguous().numpy(), g[f"out{i}"])


@pytest.mark.parametrize("name", ["decode_b3_c4_120x160", "decode_b2_c4_90x160", "decode_b1_c80_64x64"])
def test_decode_golden(name):
    g = golden(name)
    seed, B, C, H, W = [int(v) for v in g["seed"]]
    logits, size, offset, depth = decode_case_inputs(B, C, H, W, seed)
    np.testing.assert_allclose([float(t.double().sum()) for t in (logits, size, offset, depth)],
                                  g["input_checksums"], rtol=1e-10)
    nms = oracle.heatmap_nms(torch.sigmoid(logits), 3)
    np.testing.assert_array_equal(nms.numpy(), g["nms"])
    idx, lab, score = oracle.heatmap_detect(nms, 100)
    np.testing.assert_array_equal(idx.numpy(), g["index"])
    np.testing.assert_array_equal(lab.numpy(), g["label"])
    np.testing.assert_array_equal(score.numpy(), g["score"])
    in_h, in_w, ds = [int(v) for v in g["meta"]]

    class P:
        pass
    pred = P()
    pred.heatmap, pred.size, pred.offset, pred.depth = logits, size, offset, depth
    for thr in (0.05, 0.3, 0.9):
        got = oracle.decode(pred, in_h, in_w, ds, 100, thr)
        _check_records(got, g[f"decode_thr{thr}"], has_depth=True)
    pred.depth = None
    _check_records(oracle.decode(pred, in_h, in_w, ds, 100, 0.3), g["decode_nodepth_thr0.3"], has_depth=False)


def _check_records(got, ref, has_depth):
    B, K, _ = ref.shape
    for b in range(B):
        n_ref = int(np.nansum(ref[b, :, 7]))
        assert len(got[b]) == n_ref
        for i, d in enumerate(got[b]):
            row = [d[0], d[1], d[2], d[3], d[4], d[5], d[6] if has_depth else np.nan]
            np.testing.assert_array_equal(np.array(row, dtype=np.float64), ref[b, i, :7])


def _check_detcmp_self(g):
    """tests/golden/detcmp.py on the reference's own records: full agreement at any drift."""
    from detcmp import peak_parity
    ref = g["decode_k100"]
    B, K = g["decode_k100_index"].shape
    rec = np.zeros((B, K, 10))
    rec[..., :6] = ref[..., :6]
    rec[..., 7] = g["decode_k100_index"]
    for tol in (1e-6, 1e-3):
        pp = peak_parity(rec, g["heatmap"], g["decode_k100_index"], ref, tol)
        assert pp["agreement"] == 1.0 and pp["determined_found"] == pp["determined"] and pp["extra_ok"]
        assert pp["max_score_err"] == 0.0 and pp["max_box_err"] == 0.0
    # a swapped-out determined peak is caught
    if K > 1:
        bad = rec.copy()
        bad[0, 0, 7] = -1
        pp = peak_parity(bad, g["heatmap"], g["decode_k100_index"], ref, 1e-9)
        assert pp["determined_found"] == pp["determined"] - 1 and not pp["extra_ok"]


@pytest.mark.parametrize("name", [c for c in models_index()])
def test_forward_golden(name):
    case = case_by_name(name)
    if case["in_h"] * case["in_w"] * max(case["channels"]) ** 2 > 2e8:
        pytest.importorskip("torch")  # full-width 480x640 case: ~0.5 s on 8 threads, still run
    sd = case_state_dict(name)
    img = case_input(name)
    with torch.no_grad():
        pred = oracle.centernet_forward(sd, img, case["heights"], case["downsamples"], case_flags(case))
    g = golden(f"model_{name}")
    for f in FIELDS:
        t = getattr(pred, f)
        if f in g.files:
            np.testing.assert_array_equal(t.contiguous().numpy(), g[f], err_msg=f)
        else:
            assert t is None
    for thr in (0.05, 0.3):
        got = oracle.decode(pred, case["in_h"], case["in_w"], case["downsamples"], 20, thr)
        _check_records(got, g[f"decode_thr{thr}"], has_depth=pred.depth is not None)
    got = oracle.decode(pred, case["in_h"], case["in_w"], case["downsamples"], 100, 0.0)
    _check_records(got, g["decode_k100"], has_depth=pred.depth is not None)
    _check_detcmp_self(g)
    if case_flags(case)["keypoints"]:
        ratio = 2 ** case["downsamples"]
        kd = oracle.decode_keypoints(pred, case["in_h"] // ratio, case["in_w"] // ratio, keypoint_owner(case),
                                     10, 50, 0.05, 0.05)
        ref = g["decode_keypoints"]
        for b in range(ref.shape[0]):
            assert len(kd[b]) == int(np.nansum(ref[b, :, 6]))
            for i, d in enumerate(kd[b]):
                row = [d["label"], d["score"], d["y"], d["x"], d["h"], d["w"], 1.0]
                for j in range(len(d["keypoints"])):
                    if d["keypoints"][j] is None:
                        row += [np.nan] * 5
                    else:
                        row += [*d["keypoints"][j], d["keypoint_scores"][j], *d["keypoint_affinities"][j]]
                np.testing.assert_array_equal(np.array(row, dtype=np.float64), ref[b, i])


# ---- CenterpointDLA34 ----
from helpers import dla34_index, dla34_state_dict, dla34_input  # noqa: E402
from oracle.ref_dla34 import centerpoint_dla34_forward, deform_conv2d  # noqa: E402


@pytest.mark.parametrize("name", list(dla34_index()))
def test_dla34_forward_golden(name):
    """Oracle == reference CenterpointDLA34 (with the DCNv2 restatement plugged in, see
    gen_golden_dla34.py). Not bit-exact on every case: the reference's in-place `+=` and
    torch's thread-split reductions differ at the last ulp, so 1e-6 relative."""
    entry = dla34_index()[name]
    case = entry["case"]
    sd = {k[len("model."):]: v for k, v in dla34_state_dict(name).items()}
    flags = dict(keypoints=case["objects"].get("keypoints_per_label", 0) > 0)
    with torch.no_grad():
        pred = centerpoint_dla34_forward(sd, dla34_input(name), flags, len(entry["head_channels"]))
    g = golden(f"dla34_{name}")
    for f in FIELDS:
        t = getattr(pred, f)
        if f in g.files:
            ref = g[f]
            np.testing.assert_allclose(t.contiguous().numpy(), ref, rtol=0, atol=1e-6 * max(1.0, np.abs(ref).max()),
                                       err_msg=f)
        else:
            assert t is None
    flat = {int(i) for i in g["decode_k100_index"][0]}
    assert len(flat) == 100
    _check_detcmp_self(g)


def test_deform_conv2d_kat():
    """Derived known answers for the DCNv2 restatement (parity otherwise unpinned): zero
    offsets + unit mask == conv2d; a constant integer offset == conv2d of the shifted input
    (interior pixels); mask scales each tap."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 8, 13, 15, generator=g, dtype=torch.float64)
    w = torch.randn(5, 8, 3, 3, generator=g, dtype=torch.float64)
    b = torch.randn(5, generator=g, dtype=torch.float64)
    off = torch.zeros(2, 18, 13, 15, dtype=torch.float64)
    m = torch.ones(2, 9, 13, 15, dtype=torch.float64)
    torch.testing.assert_close(deform_conv2d(x, off, m, w, b), F.conv2d(x, w, b, 1, 1), rtol=1e-12, atol=1e-12)
    off[:, 0::2] = 1.0   # dy
    off[:, 1::2] = -2.0  # dx
    xs = torch.zeros_like(x)
    xs[:, :, :-1, 2:] = x[:, :, 1:, :-2]
    got = deform_conv2d(x, off, m, w, b)[:, :, 1:-2, 3:-1]
    torch.testing.assert_close(got, F.conv2d(xs, w, b, 1, 1)[:, :, 1:-2, 3:-1], rtol=1e-12, atol=1e-12)
    # half-pixel offset = mean of the two neighbours; mask 0.5 halves the tap
    off.zero_()
    off[:, 1::2] = 0.5
    m.fill_(0.5)
    xa = 0.5 * (x + torch.cat([x[:, :, :, 1:], torch.zeros_like(x[:, :, :, :1])], 3))
    # (column 0 differs by design: its left tap samples x = -0.5, half of x[0], not padding)
    torch.testing.assert_close(deform_conv2d(x, off, m, w, b)[..., 1:], F.conv2d(0.5 * xa, w, b, 1, 1)[..., 1:],
                               rtol=1e-12, atol=1e-12)
