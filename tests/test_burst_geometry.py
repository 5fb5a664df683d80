"""conv_burst.hip's LDS addressing, checked on the host (no GPU) through the library's own plan
(tv_diag_burst_plan -> conv_burst_plan + conv_burst_lds_extent, the kernel's index arithmetic
restated next to the kernel): for the layer geometries the engine hands it (3x3 windows at every
pyramid level, the fused stride-2 1x1 residual, Roots of 3 children, a two-plane 256-channel input)
every LDS byte the kernel touches lies inside the launch's dynamic LDS, and a geometry whose staging
would not fit 160 KiB is refused (an out-of-range LDS access faults the GPU on gfx950)."""
import ctypes

from tauv_vision_amd import _lib

LDS_MAX = 160 * 1024


def _plan(Ho, Wo, segs, N=128, B=2):
    """segs: (C, k, stride) per segment; a 3x3 segment is at the output size, a 1x1 at its stride."""
    geom = []
    for C, k, st in segs:
        H, W = (Ho, Wo) if k == 3 else ((Ho - 1) * st + 1, (Wo - 1) * st + 1)
        geom += [H, W, C, C, k, st]
    g = (ctypes.c_int32 * len(geom))(*geom)
    out = (ctypes.c_int32 * 4)()
    _lib.check(_lib.lib().tv_diag_burst_plan(g, len(segs), B, Ho, Wo, N, out), "burst plan")
    return list(out)


def test_burst_lds_extent_within_launch_lds():
    n = 0
    for Ho, Wo in [(15, 20), (4, 5), (8, 10), (30, 40), (60, 80), (2, 3), (1, 1), (7, 9), (33, 17), (45, 80),
                   (69, 69)]:
        for segs in ([(128, 3, 1)], [(128, 3, 1), (128, 1, 2)], [(128, 1, 1)] * 3, [(256, 1, 1), (128, 1, 1)],
                     [(256, 3, 1)]):
            ok, lds, end, need = _plan(Ho, Wo, segs)
            nk16 = sum(k * k * C // 16 for C, k, _ in segs)  # <= 4 waves x 20 register-resident k-steps
            if need <= LDS_MAX and nk16 <= 80:
                assert ok, (Ho, Wo, segs, need)
                assert 0 < end <= lds <= LDS_MAX, (Ho, Wo, segs, end, lds)
                n += 1
            else:
                assert not ok, (Ho, Wo, segs, need)
    assert n >= 35


def test_burst_refuses_what_does_not_fit():
    # a 120x160 window of a 256-channel input: ~180 KiB of staging
    ok, lds, end, need = _plan(120, 160, [(256, 3, 1), (128, 1, 2)])
    assert need > LDS_MAX and not ok and lds == 0


def test_burst_round5_fault_geometry():
    """the geometry that faulted while the kernel was written (round 5): B = 2, 15x20, one
    128-channel 3x3 segment (tests/test_gpu_conv_burst.py runs it on the GPU)"""
    ok, lds, end, need = _plan(15, 20, [(128, 3, 1)], N=128, B=2)
    assert ok and end <= lds
