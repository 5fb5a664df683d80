# The secondary bench lines: DLA34 (GPU tests + bench line + rocprofv3 kernel stats) and YOLACT
# (bench line + kernel stats). Outputs under gpurun_out/<tag>/.
set -e
O=gpurun_out/${1:-models}; mkdir -p $O/prof_dla $O/prof_yolact
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_dla34.py -x -q --timeout 200 --timeout-method thread > $O/tests_dla.log 2>&1 && echo DLA_TESTS_OK || { echo DLA_TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests_dla.log | head; tail -20 $O/tests_dla.log; exit 1; }
BENCH_PROFILE_OUT=$O/ops_dla34.json timeout -k 10 400 python bench.py --model dla34 --cpu-seconds 10 > $O/bench_dla34.log 2>&1 && echo DLA_BENCH_OK || { echo DLA_BENCH_FAIL; tail -20 $O/bench_dla34.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dla -o rprof_dla34 --output-format csv -- python bench.py --model dla34 --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-extras > $O/prof_dla.log 2>&1 && echo DLA_PROF_OK
timeout -k 10 300 python bench.py --model yolact --cpu-seconds 5 > $O/bench_yolact.log 2>&1 && echo YOLACT_BENCH_OK || { echo YOLACT_BENCH_FAIL; tail -20 $O/bench_yolact.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_yolact -o rprof_yolact --output-format csv -- python bench.py --model yolact --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_yolact.log 2>&1 && echo YOLACT_PROF_OK
python - $O <<'PY'
import json, sys
O = sys.argv[1]
for m in ("dla34", "yolact"):
    d = json.loads(open(f"{O}/bench_{m}.log").read().strip().splitlines()[-1])
    print(m, d["value"], d["unit"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"], "e2e", d.get("e2e_frac_of_peak"))
PY
