# B=1 graph replay kernel trace (R18 fp16): per-kernel time and dispatch gaps
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/b1 -o t -- python tools/b1_graph.py fp16 20 > $O/b1.log 2>&1 || { echo FAIL; tail $O/b1.log; exit 1; }
f=$(find $O/b1 -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py $f 1100
python - $f <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))[-110:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %7.1f %s" % ((s - t0) / 1e3, (e - s) / 1e3, r["Kernel_Name"].split("(")[0][:60]))
PY
