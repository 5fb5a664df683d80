# DLA34 + full GPU tests, then the dla34 bench line (no extras) and its per-op profile
set -e
O=gpurun_out/${1:-dq}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py --model dla34 --no-cpu-baseline --no-b1 --no-extras > $O/bench_dla.log 2>&1 && echo BENCH_OK || { echo BENCH_FAIL; tail -20 $O/bench_dla.log; exit 1; }
python - $O <<'PY'
import json, sys
O = sys.argv[1]
d = json.loads(open(O + "/bench_dla.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "e2e", d["e2e_frac_of_peak"], "frac", d["roofline"]["frac"])
for k, v in sorted(d["roofline"]["per_kernel"].items(), key=lambda kv: -kv[1]["ms"])[:12]:
    print(f'{v["ms"]:7.3f} ms {v["launches"]:3d} {v["tflops"]:8.1f} TF/s  {k}')
PY
