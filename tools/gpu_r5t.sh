# Decode: GPU parity tests, timing probe, and a kernel-trace profile of the bench configuration.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_parity_lowp.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python tools/decode_bench.py > $O/bench.log 2>&1 && cat $O/bench.log | grep -v amdgpu.ids || { echo BENCH_FAIL; tail $O/bench.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python tools/decode_bench.py --only > $O/prof.log 2>&1 || { echo PROF_FAIL; tail $O/prof.log; exit 1; }
f=$(ls $O/prof/*/p_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "peak" in r["Name"] or "select" in r["Name"] or "merge" in r["Name"]:
        print(r["Name"][:60], r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3), "min us %.2f" % (float(r["MinNs"]) / 1e3))
PY
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof1 -o p --output-format csv -- python tools/decode_bench.py --only1 > $O/prof1.log 2>&1 || { echo PROF1_FAIL; tail $O/prof1.log; exit 1; }
f=$(find $O/prof1 -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "peak" in r["Name"]:
        print("B=1", r["Name"][:40], r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3), "min us %.2f" % (float(r["MinNs"]) / 1e3))
PY
for s in "a:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" "b:SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"; do
  n=${s%%:*}; c=${s#*:}
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex peak -d $O/pmc -o $n --output-format csv -- python tools/decode_bench.py --only > $O/pmc_$n.log 2>&1 || { echo "PMC_$n FAIL"; tail -5 $O/pmc_$n.log; exit 1; }
done
python - $O/pmc <<'PY'
import csv, sys, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in sorted(v.items())})
PY
