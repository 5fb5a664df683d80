"""conv_burst.hip's LDS addressing on the host (no GPU): for the layer geometries the engine hands
it (3x3 windows at every pyramid level, the fused stride-2 1x1 residual, Roots of 3 children, a
two-plane 256-channel input), every staged window pixel maps to the input pixel a tap reads and every
LDS access stays inside the launch's dynamic LDS — on gfx950 an out-of-range LDS read faults."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import burst_bounds  # noqa: E402


def test_burst_lds_addressing_in_range():
    n = 0
    for Ho, Wo in [(15, 20), (4, 5), (8, 10), (30, 40), (60, 80), (2, 3), (1, 1), (7, 9), (33, 17), (69, 69)]:
        for segs in ([(128, 0, 1, Ho, Wo)], [(128, 0, 1, Ho, Wo), (128, 1, 2, 2 * Ho, 2 * Wo)],
                     [(128, 1, 1, Ho, Wo)] * 3, [(256, 1, 1, Ho, Wo), (128, 1, 1, Ho, Wo)]):
            p = burst_bounds.plan(Ho, Wo, segs, 128)
            if p["lds"] <= 160 * 1024:
                assert burst_bounds.check(p)
                n += 1
    assert n >= 35
