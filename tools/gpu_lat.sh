# conv_lat A/B: its GPU tests, the full GPU suite, then R18 / DLA34 bench lines with conv_lat on
# (default) and off (TV_LAT=0), and per-op timings of one 32-frame slice. Outputs under gpurun_out/<tag>/.
set -e
O=gpurun_out/${1:-lat}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_lat.py -x -v --timeout 120 --timeout-method thread > $O/tests_lat.log 2>&1 && echo LAT_TESTS_OK || { echo LAT_TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests_lat.log | head -20; tail -30 $O/tests_lat.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
BENCH_PROFILE_OUT=$O/ops_r18.json timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > $O/bench_r18.log 2>&1 && echo R18_OK
TV_LAT=0 timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --allow-env-knobs > $O/bench_r18_off.log 2>&1 && echo R18_OFF_OK
BENCH_PROFILE_OUT=$O/ops_dla34.json timeout -k 10 300 python bench.py --model dla34 --no-extras --no-cpu-baseline > $O/bench_dla34.log 2>&1 && echo DLA_OK
TV_LAT=0 timeout -k 10 300 python bench.py --model dla34 --no-extras --no-cpu-baseline --allow-env-knobs > $O/bench_dla34_off.log 2>&1 && echo DLA_OFF_OK
python - $O <<'PY'
import json, sys
O = sys.argv[1]
for f in ("r18", "r18_off", "dla34", "dla34_off"):
    try:
        d = json.loads(open(f"{O}/bench_{f}.log").read().strip().splitlines()[-1])
        print(f, d["value"], "ms/step", d["ms_per_step"], "B1", d.get("latency_b1"))
    except Exception as e:
        print(f, "n/a", e)
PY
