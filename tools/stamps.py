"""Summarise per-block phase stamps of pipelined convs (TV_STAMPS=<prefix> + one profile()).
Record: memtime at entry, first stage landed, main loop done, end; realtime entry/end; HW_ID; XCC_ID.
Usage: python tools/stamps.py <prefix> [ops.json]"""
import glob
import json
import sys

import numpy as np


def main():
    pre = sys.argv[1]
    labels = {}
    if len(sys.argv) > 2:
        labels = {i: o["op"] for i, o in enumerate(json.load(open(sys.argv[2])))}
    for f in sorted(glob.glob(pre + "_*.bin"), key=lambda x: int(x.rsplit("_", 1)[1][:-4])):
        i = int(f.rsplit("_", 1)[1][:-4])
        a = np.fromfile(f, dtype=np.uint64).reshape(-1, 12).astype(np.int64)
        if a[:, 10].max() > 0:  # persistent kernel: per-block totals
            a = a[a[:, 0] > 0]
            st, rt = a[:, :4], a[:, 4:6]
            ghz = np.median((st[:, 3] - st[:, 0]) / np.maximum(rt[:, 1] - rt[:, 0], 1) * 0.1)
            tiles = a[:, 10]
            tot = st[:, 3] - st[:, 0]
            span_us = (rt[:, 1].max() - rt[:, 0].min()) / 100.0
            print(f"op {i:3d} persistent blocks {len(a):4d} tiles/blk {np.median(tiles):5.1f} clk {ghz:.2f}GHz "
                  f"per tile cyc: total {np.median(tot / tiles):7.0f} stall {np.median(a[:, 8] / tiles):7.0f} "
                  f"epi {np.median(a[:, 9] / tiles):6.0f} | prologue {np.median(st[:, 1] - st[:, 0]):6.0f} "
                  f"steps/tile {np.median(a[:, 11] / tiles):4.0f} span {span_us:7.1f}us "
                  f"start spread {(rt[:, 0].max() - rt[:, 0].min()) / 100.0:5.1f}us "
                  f"end spread {(rt[:, 1].max() - rt[:, 1].min()) / 100.0:5.1f}us  {labels.get(i, '')}")
            continue
        st = a[:, :4]
        rt = a[:, 4:6]
        ghz = np.median((st[:, 3] - st[:, 0]) / np.maximum(rt[:, 1] - rt[:, 0], 1) * 0.1)
        pro, main_, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
        span_us = (rt[:, 1].max() - rt[:, 0].min()) / 100.0
        busy = (rt[:, 1] - rt[:, 0]).sum() / 100.0
        # per-CU serial gaps: key = (xcc, se, sh, cu) from HW_ID (gfx9 layout)
        hw = a[:, 6]
        cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (a[:, 7] << 8)
        gaps = []
        for c in np.unique(cu):
            idx = np.where(cu == c)[0]
            o = idx[np.argsort(rt[idx, 0])]
            gaps += list((rt[o[1:], 0] - rt[o[:-1], 1]) / 100.0)
        g = np.median(gaps) if gaps else 0
        print(f"op {i:3d} blocks {len(a):6d} clk {ghz:.2f}GHz cyc med: pro {np.median(pro):7.0f} main {np.median(main_):7.0f} "
              f"epi {np.median(epi):6.0f} | span {span_us:7.1f}us blocks/CU {len(a) / max(len(np.unique(cu)), 1):5.1f} "
              f"conc {busy / span_us / len(np.unique(cu)):.2f} gap {g:5.2f}us  {labels.get(i, '')}")


if __name__ == "__main__":
    main()
