"""Host check of conv_burst.hip's LDS addressing (its window / pixel-list staging, the k-step operand
reads, the zero block, the partial tiles) for a layer geometry: every address inside the launch's
dynamic LDS. Restates conv_burst_plan() and the kernel's index arithmetic (an out-of-range LDS access
faults the GPU on gfx950)."""
import itertools
import sys

PX, NCH, PP, SLOTS, NW, SR = 64, 32, 272, 17, 4, 36
PART = PX * SR * 4


def plan(Ho, Wo, segs, N):
    """segs: list of (C, kind, stride, H, W); -> dict like BurstParams."""
    out_rows = min(Ho, (PX + Wo - 1) // Wo + 1)
    off, k16, ss = 0, 0, []
    for C, kind, st, H, W in segs:
        d = dict(C=C, kind=kind, stride=st, H=H, W=W, planes=C // 128, kbase16=k16, lds_off=off)
        if kind == 0:
            d["wrow"] = Wo + 2
            d["npix"] = (out_rows + 2) * d["wrow"]
            k16 += 9 * C // 16
        else:
            d["wrow"] = 0
            d["npix"] = PX
            k16 += C // 16
        chunks = d["planes"] * d["npix"] * SLOTS
        off += (chunks + 63) // 64 * 1024
        ss.append(d)
    zero_off = off
    off += 256
    return dict(segs=ss, nk16=k16, zero_off=zero_off, lds=max(off, NW * PART), Ho=Ho, Wo=Wo)


def check(p, B=1):
    Ho, Wo = p["Ho"], p["Wo"]
    hw = Ho * Wo
    tiles_pf = (hw + PX - 1) // PX
    lds = p["lds"]
    for t in range(tiles_pf):
        r0 = t * PX
        npx = min(PX, hw - r0)
        y_first = r0 // Wo
        wy0 = y_first - 1
        for sg in p["segs"]:
            chunks = sg["planes"] * sg["npix"] * SLOTS
            pieces = (chunks + 63) // 64
            assert sg["lds_off"] + pieces * 1024 <= lds
            if sg["kind"] == 0:  # every window pixel a staged input row/col must exist
                for pp in range(npx):
                    r = r0 + pp
                    y, x = divmod(r, Wo)
                    pos = (y - y_first) * sg["wrow"] + x
                    for dy, dx in itertools.product(range(3), range(3)):
                        q = pos + dy * sg["wrow"] + dx
                        assert q < sg["npix"], (t, pp, dy, dx, q, sg["npix"])
                        ry, cx = divmod(q, sg["wrow"])
                        assert wy0 + ry == y - 1 + dy and cx - 1 == x - 1 + dx
            # operand reads: base + off + 16 B
            for j in range(sg["kbase16"], sg["kbase16"] + (9 if sg["kind"] == 0 else 1) * sg["C"] // 16):
                kk = j - sg["kbase16"]
                cpt = sg["C"] // 16
                tap, c16 = divmod(kk, cpt)
                o = (c16 >> 3) * sg["npix"] * PP + (c16 & 7) * 32
                if sg["kind"] == 0:
                    o += ((tap // 3) * sg["wrow"] + tap % 3) * PP
                for pp in range(PX):
                    pq = pp if pp < npx else 0
                    if sg["kind"] == 0:
                        y, x = divmod(r0 + pq, Wo)
                        pos = (y - y_first) * sg["wrow"] + x
                    else:
                        pos = pq
                    a = sg["lds_off"] + pos * PP + 16 + o + 16
                    assert a <= lds, (a, lds)
    assert p["zero_off"] + 256 <= lds and NW * PART <= lds
    return True


if __name__ == "__main__":
    cases = []
    for Ho, Wo in [(15, 20), (4, 5), (8, 10), (30, 40), (60, 80), (2, 3), (1, 1), (7, 9), (33, 17), (45, 80), (69, 69)]:
        cases.append((Ho, Wo, [(128, 0, 1, Ho, Wo)]))
        cases.append((Ho, Wo, [(128, 0, 1, Ho, Wo), (128, 1, 2, 2 * Ho, 2 * Wo)]))
        cases.append((Ho, Wo, [(128, 1, 1, Ho, Wo)] * 3))
        cases.append((Ho, Wo, [(256, 1, 1, Ho, Wo), (128, 1, 1, Ho, Wo)]))
    n = 0
    for Ho, Wo, segs in cases:
        p = plan(Ho, Wo, segs, 128)
        if p["lds"] > 160 * 1024:
            continue
        check(p)
        n += 1
    print(f"{n} geometries: every LDS access in range")
