"""Static hazard check for inline-asm ds_read_b128 in the conv kernels.

The kernels read LDS fragments with inline asm (so the compiler does not drain the LDS-DMA
vmcnt in front of every LDS read); the compiler then believes the destination registers are
ready when the asm statement ends. This scans the generated gfx950 assembly linearly and
reports any instruction that reads or overwrites a destination VGPR of an ds_read still in
flight (no `s_waitcnt lgkmcnt(0)` since the read).

Usage: python tools/check_lds_asm.py <file.s> [kernel-name-substring]
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check(lines):
    """Outstanding LDS ops are retired in order by s_waitcnt lgkmcnt(N) (N youngest stay in
    flight); only inline-asm ds_reads (between ;;#ASMSTART/END) are tracked for hazards, the
    compiler's own LDS ops only occupy the queue."""
    queue = []  # [(regs or empty set)] oldest first
    issues = []
    in_asm = False
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
        m = re.search(r"lgkmcnt\((\d+)\)", line) if op == "s_waitcnt" else None
        if m:
            n = int(m.group(1))
            queue = queue[len(queue) - n:] if n < len(queue) else queue
            if n == 0:
                queue = []
            continue
        if op.startswith("s_"):
            continue
        pending = set().union(*queue) if queue else set()
        args = line[len(op):]
        if op.startswith("ds_"):
            if op.startswith("ds_read"):
                dst, src = args.split(",", 1)
                hit = regs(src) & pending
                if hit:
                    issues.append((no, raw.strip(), sorted(hit)))
                d = regs(dst)
                if d & pending:
                    issues.append((no, raw.strip() + "   [WAW]", sorted(d & pending)))
                queue.append(d if in_asm else set())
            else:
                hit = regs(args) & pending
                if hit:
                    issues.append((no, raw.strip(), sorted(hit)))
                queue.append(set())
            continue
        hit = regs(args) & pending
        if hit:
            issues.append((no, raw.strip(), sorted(hit)))
    return issues


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read().splitlines()
    fn, body, total = None, [], 0
    for i, l in enumerate(text, 1):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            fn, body = m.group(1), []
            continue
        if fn and l.strip().startswith(".Lfunc_end"):
            if want in fn:
                iss = check(body)
                total += len(iss)
                print(f"{fn}: {len(iss)} hazards")
                for it in iss[:10]:
                    print("   line", it[0], it[1], "regs", it[2])
            fn = None
        elif fn:
            body.append((i, l))
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
