"""Mean launch duration of one kernel over consecutive windows of a rocprofv3 kernel trace: separates
a bench run's phases (eager warm-up, the timed graph replays with the concurrent slices contending
for CUs, the serialised per-op profile passes, the in-situ graph replays of bench.conv_roofline),
which the --stats average mixes. Usage: python tools/trace_phases.py <kernel_trace.csv> <name substring> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 36
t0 = min(int(r["Start_Timestamp"]) for r in rows)
d = sorted((int(r["Start_Timestamp"]) - t0, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
           for r in rows if sub in r["Kernel_Name"])
print(f"{len(d)} launches of *{sub}*, windows of {n}")
for i in range(0, len(d), n):
    c = d[i:i + n]
    print(f"t = {c[0][0] / 1e6:9.1f} ms  n = {len(c):3d}  mean {sum(x[1] for x in c) / len(c):8.1f} us  "
          f"min {min(x[1] for x in c):8.1f}  max {max(x[1] for x in c):8.1f}")
