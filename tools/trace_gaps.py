"""Summarise a rocprofv3 kernel-trace CSV of graph replays: per kernel name the average duration,
and the average gap between consecutive dispatches (end -> next start) within replays."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # only the last N dispatches (steady replays)
if last:
    rows = rows[-last:]
dur = defaultdict(list)
gaps = []
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[r["Kernel_Name"].split("(")[0][:70]].append(e - s)
    if prev_end is not None:
        gaps.append(s - prev_end)
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"{len(rows)} dispatches over {span:.1f} us; busy {sum(sum(v) for v in dur.values()) / 1e3:.1f} us; "
      f"gaps sum {sum(g for g in gaps if g > 0) / 1e3:.1f} us, median gap {sorted(gaps)[len(gaps) // 2] / 1e3:.2f} us")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / 1e3:8.1f} us {len(v):4d} x {sum(v) / len(v) / 1e3:6.2f} us  {k}")
