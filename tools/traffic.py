"""HBM traffic per kernel instance from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; one
pass each, tools/prof_forward.py --iters 1 = one forward of the bench workload).

FETCH_SIZE / WRITE_SIZE are KiB. On gfx950 FETCH_SIZE counts exactly half the bytes of 16-B/lane
streaming reads of whole 128-B lines (MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE
is exact for 16-B/lane stores. Reads issued as 64-B half lines are different: calibrated on this chip
(tools/micro/halo_fetch.hip, profiles/r6/halo_fetch_calibration.txt) a 629 MB tensor read in 64-B
pieces reports FETCH_SIZE = 629 MB (the true bytes), read whole-line it reports 314.6 MB. The halo
kernels (conv3x3, conv3x3s2, convt3) move their activations — halo and residual — in exactly such
64-B pieces (32 channels of a 128-channel pixel, 4 lanes x 16 B; the weights are L2-resident), so
their FETCH_SIZE is taken x1; every other kernel x2 (fetch_factor per kernel in the output). Usage:
  python tools/traffic.py <FETCH_SIZE_counter_collection.csv> <WRITE_SIZE_counter_collection.csv> \
      --batch 64 --precision fp16 -o profiles/hbm_traffic.json
"""
import argparse
import collections
import csv
import json
import subprocess


def demangle(name):
    if not name.startswith("_Z"):
        return name
    # binutils' c++filt predates the _Float16 mangling (DF16_): demangle it as 'half' and rename
    out = subprocess.run(["c++filt", name.replace("DF16_", "Dh")], capture_output=True, text=True).stdout.strip()
    out = out.replace("half", "_Float16")
    out = out[5:] if out.startswith("void ") else out
    return out.split("(")[0]


def per_kernel(path, counter):
    acc = collections.defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = acc[demangle(r["Kernel_Name"])]
            k[0] += 1
            k[1] += float(r["Counter_Value"]) * 1024.0
    return acc


# kernels whose HBM reads are 64-B half-line pieces (LDS-DMA halo / residual chunks at an 80-B pitch)
HALF_LINE = ("tv::c3::conv3x3<", "tv::c3s2::conv3x3s2<", "tv::ct3::convt3<")


def fetch_factor(kernel):
    return 1.0 if kernel.startswith(HALF_LINE) else 2.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--batch", type=int, default=32, help="frames per launch (a B=64 forward = two 32-frame slices)")
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("-o", "--out", default="profiles/hbm_traffic.json")
    a = ap.parse_args()
    fe, wr = per_kernel(a.fetch, "FETCH_SIZE"), per_kernel(a.write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        n = max(fe[k][0], wr[k][0])
        fb, wb = fetch_factor(k) * fe[k][1], wr[k][1]
        kernels[k] = {"launches": n, "fetch_bytes": fb, "write_bytes": wb, "fetch_factor": fetch_factor(k),
                      "bytes_per_launch": (fb + wb) / max(n, 1)}
    res = {"batch": a.batch, "precision": a.precision,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one forward (tools/prof_forward.py --iters 1); "
                     "FETCH_SIZE x2 (gfx950 whole-line streams), x1 for the halo kernels' 64-B half-line reads "
                     "(tools/micro/halo_fetch.hip calibration), KiB -> bytes",
           "total_bytes": sum(v["fetch_bytes"] + v["write_bytes"] for v in kernels.values()),
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -(kv[1]["fetch_bytes"] + kv[1]["write_bytes"])):
        print(f"{v['launches']:4d} {v['fetch_bytes'] / 1e9:8.3f} GB rd {v['write_bytes'] / 1e9:8.3f} GB wr  {k}")


if __name__ == "__main__":
    main()
