"""Phase stamps of peak_select (debug variant tools/dbg/decode_st.hip, TV_LIB=...variants/dst.so):
per image the wall-clock (10 ns) of the phase boundaries, from the last record's fields."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tauv-vision_amd")]
import numpy as np
import torch
from tauv_vision_amd.decode import DeviceDecoder
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(1)
for B, K in ((64, 100), (1, 100), (64, 1)):
    logits = (torch.randn((B, 4, 120, 160), generator=g) * 2).cuda()
    size = torch.randn((B, 120, 160, 2), generator=g).cuda()
    off = torch.rand((B, 120, 160, 2), generator=g).cuda()
    d = DeviceDecoder(B, 4, 120, 160, K, dev)
    for _ in range(3):
        rec, cnt = d(logits, size, off, None, 0, 4, 480, 640, 0.0)
    torch.cuda.synchronize()
    st = rec[:, K - 1, :8].cpu().numpy().view(np.uint32).astype(np.int64)
    dl = np.diff(st, axis=1) * 10 / 1000.0  # us
    print(f"B={B} K={K} phases (us, median over images): " + " ".join(f"{x:.2f}" for x in np.median(dl, axis=0)),
          " total %.2f us" % (np.median(st[:, 7] - st[:, 0]) / 100.0) )
