# convt3 timing experiments: default, stale weights (1), stale halo (2), both (3), no MFMA (4), forced 16x16 tile
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5o; mkdir -p $O
run() { timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$1 -o run -- python tools/ct3_time.py $2 $3 $4 > $O/$1.log 2>&1 || { echo "fail $1"; tail -5 $O/$1.log; exit 1; }; }
run base tauv-vision_amd/lib/libtauv_vision_amd.so && run t16 tauv-vision_amd/lib/libtauv_vision_amd.so 16 16 && \
run c1 tauv-vision_amd/lib_c1/libtauv_vision_amd.so && run c2 tauv-vision_amd/lib_c2/libtauv_vision_amd.so && \
run c3 tauv-vision_amd/lib_c3/libtauv_vision_amd.so && run c4 tauv-vision_amd/lib_c4/libtauv_vision_amd.so
for d in base t16 c1 c2 c3 c4; do f=$(find $O/$d -name "*kernel_trace.csv" | head -1); python - "$f" "$d" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "convt3" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
a, b = d[0::2][1:], d[1::2][1:]
print(sys.argv[2], "69x69: %.1f us" % (sum(a) / len(a)), "138x138: %.1f us" % (sum(b) / len(b)))
PY
done
