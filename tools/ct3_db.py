"""Per-shape convt3 kernel durations from a rocprofv3 run of tools/ct3_time.py (sqlite output)."""
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
    fs = glob.glob(f"{d}/*.db")
    if not fs:
        continue
    con = sqlite3.connect(fs[0])
    rows = con.execute("select name, start, end from kernels where name like '%convt3%' order by start").fetchall()
    dur = [(r[2] - r[1]) / 1e3 for r in rows]
    a, b = dur[1:6], dur[7:12]
    print(d, "69x69 %.1f us (%.0f TF/s)" % (sum(a) / len(a), 179.7e3 / (sum(a) / len(a))),
          "138x138 %.1f us (%.0f TF/s)" % (sum(b) / len(b), 718.8e3 / (sum(b) / len(b))))
