"""Where one B=64 bench step's wall time goes (rocprofv3 --kernel-trace CSV of a bench run; the step between two decode launches):
per kernel family, the wall time it ran alone, the wall time shared with the other slice's
kernels (split evenly), and the idle gaps. Usage: python tools/timeline.py <kernel_trace.csv>"""
import collections
import csv
import re
import sys


def family(name):
    """kernel family of a (mangled or demangled) kernel name; conv3x3 instances keep their template
    arguments (tile width, epilogue, residual, channel fragments, waves)"""
    n = re.sub(r"^_ZN2tv", "", name)
    for key, lab in (("c3s2", "conv3x3s2"), ("conv_lat", "conv_lat"), ("conv_pipe", "conv_pipe"),
                     ("conv_burst", "conv_burst"), ("conv1x1", "conv1x1_stream"), ("stem_s2", "stem_s2"),
                     ("convt3", "convt3"), ("convt_add", "convt_add"), ("stem_conv", "stem"), ("peak_scan", "decode"),
                     ("fill_zero", "fill_zero"), ("dcn", "dcn"), ("dla::", "dla"), ("conv_small", "conv_small")):
        if key in n:
            return lab
    m = re.search(r"conv3x3<[^,]+, [^,]+, (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", n)
    if m:
        tw, act, epi, res, ni, ncb, nw = m.groups()
        return "conv3x3 tw%s epi%s res%s ni%s nw%s" % (tw, epi, res, ni, nw)
    m = re.search(r"conv3x3I(DF16_DF16_|DF16bDF16b)Li(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E(Li(\d+)E)?", n)
    if m:
        tw, act, epi, res, ni = m.group(2), m.group(3), m.group(4), m.group(5), m.group(6)
        return "conv3x3 tw%s epi%s res%s ni%s" % (tw, epi, res, ni)
    return n[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"]), r["Kernel_Name"]) for r in rows]
    ev.sort()
    # steps: delimited by the decode select kernel (one per step); take the last full step
    sel = [i for i, e in enumerate(ev) if "peak_scan" in e[3]]
    if len(sel) < 3:
        print("no steps found")
        return
    # argv[2]: which step (0-based boundary index; default 6: a graph replay of a bench run with
    # 2 eager warm-up steps before capture, then the replays, then the eager comparison steps)
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    k = min(k, len(sel) - 2)
    a, b = sel[k] + 1, sel[k + 1] + 1
    step = ev[a:b]
    t0, t1 = step[0][0], max(e[1] for e in step)
    pts = sorted({t for e in step for t in (e[0], e[1])})
    alone = collections.Counter()
    shared = collections.Counter()
    idle = 0
    for lo, hi in zip(pts, pts[1:]):
        run = [e for e in step if e[0] <= lo and e[1] >= hi]
        dt = hi - lo
        if not run:
            idle += dt
        elif len(run) == 1:
            alone[run[0][2]] += dt
        else:
            for e in run:
                shared[e[2]] += dt / len(run)
    wall = t1 - t0
    print("step wall %.3f ms, %d kernels, idle %.3f ms" % (wall / 1e6, len(step), idle / 1e6))
    fams = sorted(set(alone) | set(shared), key=lambda f: -(alone[f] + shared[f]))
    print("%-36s %9s %9s %9s %6s" % ("family", "alone ms", "shared ms", "sum ms", "share"))
    for f in fams:
        s = alone[f] + shared[f]
        print("%-36s %9.3f %9.3f %9.3f %5.1f%%" % (f, alone[f] / 1e6, shared[f] / 1e6, s / 1e6, 100 * s / wall))


if __name__ == "__main__":
    main()
