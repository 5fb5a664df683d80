# Quick measure: forward GPU tests + default bench without extras; per-kernel summary of one slice
set -e
O=gpurun_out/${1:-q}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_parity_lowp.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
BENCH_PROFILE_OUT=$O/ops.json timeout -k 10 300 python bench.py --no-cpu-baseline --no-b1 --no-extras ${BENCH_ARGS} > $O/bench.log 2>&1 && echo BENCH_OK || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
python - $O <<'PY'
import json, sys
O = sys.argv[1]
d = json.loads(open(O + "/bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for k, v in sorted(d["roofline"]["per_kernel"].items(), key=lambda kv: -kv[1]["ms"]):
    print(f'{v["ms"]:7.3f} ms {v["launches"]:3d} {v["tflops"]:8.1f} TF/s  {k}')
PY
