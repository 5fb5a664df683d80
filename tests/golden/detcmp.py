"""Detection-level comparison of device decode records against the reference's golden records.

Test / measurement infrastructure (numpy over committed fixture data; no oracle code): used
by tests/test_gpu_parity_lowp.py and by bench.py's parity leg.

The reference decode (decode.py:179-236) picks the top-K peaks of sigmoid -> 3x3 NMS. A
reduced-precision forward moves every logit by up to some drift `tol`, i.e. every score by up
to tol/4, so two scores' order is only fixed when they differ by more than tol/2 (`stol`).
A cell can be a peak under drift only if it is within stol of its strongest neighbour
("near-peak"). A reference peak p is *determined* when it beats its strongest neighbour by
more than stol AND fewer than K other near-peak cells could score at least as high as p
under drift (reference score >= score(p) - stol): then p is in the top-K for every
perturbation within `tol` and must be found, at the same cell. `peak_parity` reports:

  agreement          |GPU top-K  cap  reference top-K| / K (cells, i.e. flat indices)
  determined         reference top-K peaks whose top-K membership no drift <= tol can change
  determined_found   how many of those the GPU returned (must equal `determined`)
  extra_ok           every GPU peak outside the reference top-K is a near-peak cell whose
                     reference score is within stol of the K-th *robust* reference peak (a
                     peak beating its neighbours by more than stol stays a peak under any
                     drift; a marginal reference peak may stop being one, so the GPU's K-th
                     score is bounded below by the robust peaks only, not by the K-th peak)
  max_score_err      over matched peaks, |score_gpu - score_ref|
  max_box_err        over matched peaks, max |(y, x, h, w)_gpu - (y, x, h, w)_ref|
"""
import numpy as np


def _sigmoid(x):
    x = x.astype(np.float32)
    return (np.float32(1.0) / (np.float32(1.0) + np.exp(-x))).astype(np.float32)


def _neighbour_max(sig):
    """max over the 8 neighbours (implicit -inf padding, max_pool2d semantics)."""
    B, C, H, W = sig.shape
    p = np.full((B, C, H + 2, W + 2), -np.inf, dtype=np.float32)
    p[:, :, 1:-1, 1:-1] = sig
    m = np.full_like(sig, -np.inf)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy or dx:
                m = np.maximum(m, p[:, :, 1 + dy:1 + dy + H, 1 + dx:1 + dx + W])
    return m


def peak_parity(got_records, ref_heat_logits, ref_index, ref_records, tol):
    """got_records [B,K,10] (tv_decode layout), ref_heat_logits [B,C,H,W] (reference
    Prediction.heatmap), ref_index [B,K] (reference flat peaks), ref_records [B,K,8]
    (gen_golden._pack_dets of decode(K, thr=0)); tol = logit drift bound."""
    got_records = np.asarray(got_records, dtype=np.float64)
    B, K = ref_index.shape
    sig = _sigmoid(ref_heat_logits)
    nb = _neighbour_max(sig)
    flat_sig = sig.reshape(B, -1)
    flat_nb = nb.reshape(B, -1)
    stol = 2.0 * 0.25 * tol  # sigmoid' <= 1/4: a logit drift of tol moves a score by <= tol/4
    out = dict(agreement=0.0, determined=0, determined_found=0, extra_ok=True, max_score_err=0.0,
               max_box_err=0.0, matched=0, K=K)
    agree = 0
    for b in range(B):
        robust = np.sort(flat_sig[b][flat_sig[b] - flat_nb[b] > stol])[::-1]
        s_k = float(robust[K - 1]) if robust.size >= K else -np.inf
        # scores of every cell that could be a peak under drift, ascending
        cand = np.sort(flat_sig[b][flat_nb[b] - flat_sig[b] <= stol])
        got_idx = got_records[b, :, 7].astype(np.int64)
        ref_set = {int(i): r for r, i in enumerate(ref_index[b])}
        got_set = {int(i): r for r, i in enumerate(got_idx)}
        agree += len(set(ref_set) & set(got_set))
        for i, r in ref_set.items():
            rivals = cand.size - int(np.searchsorted(cand, flat_sig[b, i] - stol, side="left")) - 1
            det = rivals < K and flat_sig[b, i] - flat_nb[b, i] > stol
            if det:
                out["determined"] += 1
                out["determined_found"] += int(i in got_set)
            if i in got_set:
                g = got_records[b, got_set[i]]
                ref = ref_records[b, r]
                out["matched"] += 1
                out["max_score_err"] = max(out["max_score_err"], abs(g[1] - ref[1]))
                out["max_box_err"] = max(out["max_box_err"], float(np.max(np.abs(g[2:6] - ref[2:6]))))
        for i in got_set:
            if i in ref_set:
                continue
            near_cut = flat_sig[b, i] >= s_k - stol
            near_peak = flat_nb[b, i] - flat_sig[b, i] <= stol
            out["extra_ok"] &= bool(near_cut and near_peak)
    out["agreement"] = agree / float(B * K)
    return out

