"""Static hazard check for the inline-asm 16x16x32 MFMAs of conv3x3's K16 body.

conv3x3_kernel.h issues the main-loop v_mfma_f32_16x16x32_{f16,bf16} as asm statements with the
accumulator tied to src C (mfma16_asm) and places the hazards by hand: inside the loop an
accumulator's only reader is the next MFMA taking it whole as C; the epilogue's first reader sits
behind mfma16_drain() (s_nop 7; s_nop 4). LLVM's hazard recognizer does not see these asm
statements as MFMAs, so if the compiler ever put a VALU copy or read of an accumulator between
them (a register-allocation change, a compiler upgrade) it would insert no wait states and the
results would silently go wrong. This scans the generated gfx950 assembly linearly and reports
every instruction outside the asm MFMAs that references an accumulator register of an asm MFMA
issued since the last drain.

Usage: python tools/check_mfma_asm.py <file.s> [kernel-name-substring]
(`hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip -S --cuda-device-only csrc/conv3x3_n4.hip`;
tests/test_isa_checks.py runs it on the K16 instances.)
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
MFMA16 = re.compile(r"^v_mfma_f32_16x16x32_(f16|bf16)\s+(\S+?),")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check(lines):
    """Returns (issues, asm_mfmas, drains) for one function body [(line_no, text)]."""
    pending = set()  # accumulator registers of asm MFMAs since the last drain
    issues, n_mfma, n_drain = [], 0, 0
    in_asm = False
    prev_nop7 = False
    for no, raw in lines:
        if "#ASMSTART" in raw:
            in_asm = True
            continue
        if "#ASMEND" in raw:
            in_asm = False
            continue
        line = raw.split(";")[0].strip()
        if not line or line.endswith(":") or line.startswith("."):
            continue
        op = line.split()[0]
        if in_asm:
            m = MFMA16.match(line)
            if m:
                pending |= regs(m.group(2))
                n_mfma += 1
            if op == "s_nop":
                if line.endswith(" 7"):
                    prev_nop7 = True
                    continue
                if line.endswith(" 4") and prev_nop7:
                    pending = set()
                    n_drain += 1
            prev_nop7 = False
            continue
        prev_nop7 = False
        if op.startswith("s_"):
            continue  # scalar / control: no VGPR operands
        hit = regs(line[len(op):]) & pending
        if hit:
            issues.append((no, raw.strip(), sorted(hit)))
    return issues, n_mfma, n_drain


def scan(path, want=""):
    """{function: (issues, asm_mfmas, drains)} of the functions whose name contains `want`."""
    text = open(path).read().splitlines()
    out = {}
    fn, body = None, []
    for i, l in enumerate(text, 1):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            fn, body = m.group(1), []
            continue
        if fn and l.strip().startswith(".Lfunc_end"):
            if want in fn:
                out[fn] = check(body)
            fn = None
        elif fn:
            body.append((i, l))
    return out


def main():
    res = scan(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    total = 0
    for fn, (iss, n, d) in res.items():
        if not n:
            continue
        total += len(iss)
        print(f"{fn}: {n} asm MFMAs, {d} drains, {len(iss)} hazards")
        for it in iss[:10]:
            print("   line", it[0], it[1], "regs", it[2])
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
