"""Static checks of the generated gfx950 code of the hand-scheduled conv3x3 bodies (CPU: hipcc
cross-compiles; no GPU needed).

conv3x3_kernel.h issues its fragment LDS reads (ds_read_b128) and, in the 16x16x32 (K16) body,
its MFMAs as inline asm, with the waits and hazards placed by hand; the compiler does not see
either as what they are. Two linear scans of the assembly of the 128-channel-input instances
(conv3x3_n4.hip, which holds the dominant K16 layer) guard those hand placements:
  * tools/check_mfma_asm.py: no instruction outside the asm MFMAs touches an accumulator of an
    asm MFMA between it and the next mfma16_drain() (s_nop 7; s_nop 4) — the advisor's ISA check;
  * tools/check_lds_asm.py: no instruction reads or overwrites the destination of an asm
    ds_read still in flight (no lgkmcnt wait since the read).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def conv3x3_n4_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "conv3x3_n4.s"
    src = os.path.join(ROOT, "tauv-vision_amd", "csrc", "conv3x3_n4.hip")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-S", "--cuda-device-only",
                    src, "-o", str(out)], check=True, capture_output=True, timeout=600)
    return str(out)


def test_k16_asm_mfma_accumulators_untouched_until_drain(conv3x3_n4_asm):
    import check_mfma_asm
    res = {fn: r for fn, r in check_mfma_asm.scan(conv3x3_n4_asm).items() if r[1] > 0}
    # the K16 body runs in the plain-epilogue 128-channel-tile instances (fp16 and bf16, each
    # activation and tile width): all of them issue asm MFMAs and drain before their epilogue
    assert len(res) >= 4, sorted(res)
    for fn, (issues, n_mfma, n_drain) in res.items():
        assert n_drain >= 1, fn
        assert not issues, (fn, issues[:5])


def test_asm_lds_reads_waited_before_use(conv3x3_n4_asm):
    import re
    import check_lds_asm
    text = open(conv3x3_n4_asm).read().splitlines()
    fn, body, checked = None, [], 0
    for i, l in enumerate(text, 1):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            fn, body = m.group(1), []
            continue
        if fn and l.strip().startswith(".Lfunc_end"):
            if "conv3x3" in fn:
                issues = check_lds_asm.check(body)
                assert not issues, (fn, issues[:5])
                checked += 1
            fn = None
        elif fn:
            body.append((i, l))
    assert checked >= 4


def test_mfma_checker_flags_an_accumulator_touch():
    """The scan itself: a VALU read of an asm MFMA's accumulator before the drain is reported,
    the same read after s_nop 7; s_nop 4 is not."""
    import check_mfma_asm
    body = [(1, "\t;;#ASMSTART"), (2, "\tv_mfma_f32_16x16x32_f16 v[0:3], v[8:11], v[12:15], v[0:3]"),
            (3, "\t;;#ASMEND"), (4, "\tv_mov_b32_e32 v20, v2"), (5, "\t;;#ASMSTART"), (6, "\ts_nop 7"),
            (7, "\ts_nop 4"), (8, "\t;;#ASMEND"), (9, "\tv_add_f32_e32 v21, v1, v3")]
    issues, n_mfma, n_drain = check_mfma_asm.check(body)
    assert n_mfma == 1 and n_drain == 1
    assert [i[0] for i in issues] == [4]
