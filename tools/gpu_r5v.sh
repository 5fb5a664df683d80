# single-launch decode: GPU decode + parity tests, timing probe, B=64 / B=1 kernel traces
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_parity_lowp.py tests/test_gpu_replay_b1.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python tools/decode_bench.py > $O/bench.log 2>&1 && grep -v amdgpu.ids $O/bench.log || { echo BENCH_FAIL; tail $O/bench.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python tools/decode_bench.py --only > $O/prof.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof1 -o p --output-format csv -- python tools/decode_bench.py --only1 > $O/prof1.log 2>&1
for d in prof prof1; do f=$(find $O/$d -name "*kernel_stats.csv" | head -1); python - "$f" $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "peak" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3), "min us %.2f" % (float(r["MinNs"]) / 1e3))
PY
done
timeout -k 10 120 python tools/dec_stamps.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 > $O/bench.log 2>&1; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], {k:v['ms_per_frame'] for k,v in d['latency_b1'].items()}, d['roofline']['frac'])
"
