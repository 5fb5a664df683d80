# Generic A/B: GPU test suite, then R18 and DLA34 bench lines for the default build and with the
# environment knob assignment given as $2 (e.g. TV_PRIO=0). Outputs under gpurun_out/<tag>/.
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
KNOB=${2:-TV_PRIO=0}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
for m in r18 dla34; do
  BENCH_PROFILE_OUT=$O/ops_$m.json timeout -k 10 300 python bench.py --model $m --no-extras --no-cpu-baseline > $O/bench_$m.log 2>&1 && echo ${m}_OK
  env $KNOB timeout -k 10 300 python bench.py --model $m --no-extras --no-cpu-baseline --allow-env-knobs > $O/bench_${m}_knob.log 2>&1 && echo ${m}_KNOB_OK
done
python - $O <<'PY'
import json, sys
O = sys.argv[1]
for f in ("r18", "r18_knob", "dla34", "dla34_knob"):
    d = json.loads(open(f"{O}/bench_{f}.log").read().strip().splitlines()[-1])
    b1 = {k: v["ms_per_frame"] for k, v in d.get("latency_b1", {}).items()}
    print(f, d["value"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"], "B1", b1)
PY
