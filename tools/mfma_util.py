"""MFMA utilisation and held clock per kernel instance from one rocprofv3 PMC pass
(GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES; tools/prof_forward.py --iters 1).

Per dispatch (rocprofv3 serialises dispatches while it collects counters):
  clock      = GRBM_GUI_ACTIVE / 8 / duration        (GRBM is summed over the 8 XCDs; reads high
                                                      below ~0.3 ms: MI355X_MICROARCH.md DVFS give-back)
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  frac@2.4   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x 2.4 GHz x duration): the busy fraction priced at the
               nominal clock, the same quantity as bench.py's roofline.frac when the kernel runs only
               dense MFMAs of the timed dtype
Usage: python tools/mfma_util.py <counter_collection.csv> [-o out.json]
"""
import argparse
import collections
import csv
import json

SIMDS = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("-o", default="")
    a = ap.parse_args()
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(a.csv)):
        d = disp[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    agg = collections.OrderedDict()
    for d in disp.values():
        if "GRBM_GUI_ACTIVE" not in d or "SQ_VALU_MFMA_BUSY_CYCLES" not in d:
            continue
        k = agg.setdefault(d["name"], {"launches": 0, "ns": 0, "grbm": 0.0, "mfma": 0.0, "sqbusy": 0.0})
        k["launches"] += 1
        k["ns"] += d["ns"]
        k["grbm"] += d["GRBM_GUI_ACTIVE"]
        k["mfma"] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
        k["sqbusy"] += d.get("SQ_BUSY_CYCLES", 0.0)
    out = {}
    for name, k in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        if k["mfma"] <= 0:
            continue
        cyc = k["grbm"] / 8
        out[name] = {"launches": k["launches"], "ms": round(k["ns"] / 1e6, 4),
                     "clock_GHz": round(cyc / k["ns"], 3),
                     "mfma_busy": round(k["mfma"] / (SIMDS * cyc), 4),
                     "mfma_busy_at_2p4GHz": round(k["mfma"] / (SIMDS * 2.4 * k["ns"]), 4),
                     "mfma_busy_cycles_per_launch": k["mfma"] / k["launches"]}
    for n, v in list(out.items())[:14]:
        print(f"{v['ms']:8.3f} ms x{v['launches']:3d}  clock {v['clock_GHz']:.2f} GHz  mfma busy {v['mfma_busy']:.3f}"
              f"  (@2.4 GHz {v['mfma_busy_at_2p4GHz']:.3f})  {n[:90]}")
    if a.o:
        json.dump({"source": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES, "
                             "tools/prof_forward.py --iters 1 (dispatches serialised by the profiler)",
                   "kernels": out}, open(a.o, "w"), indent=1)


if __name__ == "__main__":
    main()
