"""Debug helper: the DLA34 B=64 detection-parity case with per-extra-peak details."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tauv-vision_amd"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch
import test_gpu_parity_lowp as T
from detcmp import _sigmoid, _neighbour_max
from recipe import seeded_u8_frames
from tauv_vision_amd.decode import DeviceDecoder

arch, name, precision, B = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
model, mc, case, g = T._build(arch, name, precision)
H, W = case["in_h"], case["in_w"]
frame = seeded_u8_frames(1, H, W, seed=case["seed"])
frames = seeded_u8_frames(B, H, W, seed=999)
for s in T.SLOTS[B]:
    frames[s] = frame[0]
with torch.no_grad():
    pred = model.forward_frames(frames.cuda())
C, Ho, Wo = pred.heatmap.shape[1:]
dec = DeviceDecoder(B, C, Ho, Wo, 100, pred.heatmap.device)
rec, _ = dec(pred.heatmap, pred.size, pred.offset, None, 0, mc.downsample_ratio, H, W, 0.0)
rec = rec.cpu().numpy()
ref = g["heatmap"][:1]
sig = _sigmoid(ref); nb = _neighbour_max(sig)
peaks = np.where(sig >= nb, sig, 0).reshape(-1)
s_k = np.sort(peaks)[::-1][99]
for s in T.SLOTS[B]:
    gh = pred.heatmap[s:s + 1].cpu().numpy()
    hm = float(np.abs(gh - ref).max())
    gs = _sigmoid(gh); gnb = _neighbour_max(gs)
    stol = 0.5 * hm
    idx = rec[s, :, 7].astype(np.int64)
    refset = set(int(i) for i in g["decode_k100_index"][0])
    print(f"slot {s}: hm_err {hm:.3e} stol {stol:.3e} s_k {s_k:.7f}")
    for r, i in enumerate(idx):
        if i in refset:
            continue
        print(f"  extra rank {r} idx {i}: gpu rec score {rec[s, r, 1]:.7f} gpu sig {gs.reshape(-1)[i]:.7f} gpu nb {gnb.reshape(-1)[i]:.7f}"
              f" ref sig {sig.reshape(-1)[i]:.7f} ref nb {nb.reshape(-1)[i]:.7f} near_cut {sig.reshape(-1)[i] >= s_k - stol}"
              f" near_peak {nb.reshape(-1)[i] - sig.reshape(-1)[i] <= stol}")
