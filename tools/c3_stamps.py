"""Where a conv3x3 k-step spends its cycles: run one forward slice with the stamp build of the
library (make BUILD=build_s9 LIBDIR=lib_s9 EXTRA=-DTV_C3_EXP=9; TV_LIB=.../lib_s9/...) and print
the per-wave cycle buckets of the chosen ops (shares, not lengths: the stamps add fences).
Usage: TV_LIB=<lib_s9> python tools/c3_stamps.py --match output_layers.0.0 [--batch 32]
The fused stem (stem_s2.hip) has its own buckets: --match block_layers.0.conv1 --kernel tv::ss2::"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

NAMES = ["barrier (taps 0-7)", "first half (+H1 drain)", "second half (+H0 drain)", "epilogue", "prologue", "k-steps",
         "tap-8 halo vmcnt wait", "tap-8 barrier"]
TIME = [0, 1, 2, 3, 4, 6, 7]
SS2_NAMES = ["block barrier", "stem phase", "k-step barrier (+ first reads)", "k-step halves", "staging under k-steps",
             "epilogue", "prologue / tile end", "k-steps"]
SS2_TIME = [0, 1, 2, 3, 4, 5, 6]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--model", default="r18")
    ap.add_argument("--match", default="ida_up_reverse.output_layers.0.0")
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--kernel", default="tv::c3::conv3x3<")
    a = ap.parse_args()
    knobs = bench.env_knobs()
    from tauv_vision_amd import _lib
    from tauv_vision_amd.engine import set_diagnostic_knobs
    if "TV_LIB" in knobs:
        _lib.set_library_path(knobs.pop("TV_LIB"))
    dev = torch.device("cuda", 0)
    frames = torch.randint(0, 256, (a.batch, 480, 640, 3), device=dev, dtype=torch.uint8)
    model, oc, sd = bench.build_model(a.precision, dev, a.model)
    eng = model.engine(dev, 480, 640)
    ops = eng.profile(frames, eng.alloc_out(a.batch))
    sel = [i for i, o in enumerate(ops) if a.match in o[0] and o[3].startswith(a.kernel)]
    names, time, cnt = (SS2_NAMES, SS2_TIME, 7) if a.kernel.startswith("tv::ss2") else (NAMES, TIME, 5)
    res = []
    for i in sel[:4]:
        buf = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
        set_diagnostic_knobs(dict(knobs, TV_C3_STAMPS=f"{i}:{buf.data_ptr()}"))
        m2, _, _ = bench.build_model(a.precision, dev, a.model)
        e2 = m2.engine(dev, 480, 640)
        prof = e2.profile(frames, e2.alloc_out(a.batch))
        torch.cuda.synchronize()
        v = buf.view(256 * 8, 8).cpu()
        used = v[v[:, cnt] > 0].double()
        tot = used[:, time].sum(1)
        steps = float(used[:, cnt].mean())
        res.append({"op": ops[i][0], "kernel": ops[i][3], "ms_stamped": round(prof[i][1], 4), "waves": int(used.shape[0]),
                    "share": {names[k]: round(float(used[:, k].sum() / tot.sum()), 4) for k in time},
                    "k_steps_per_wave": steps,
                    "cycles_per_kstep": round(float((tot / used[:, cnt]).mean()), 1),
                    "bucket_cycles_per_kstep": {names[k]: round(float((used[:, k] / used[:, cnt]).mean()), 1)
                                                for k in time}})
        set_diagnostic_knobs({})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
