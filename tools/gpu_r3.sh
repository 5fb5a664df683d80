# Round-3 measurement call: GPU tests (main suite, then the DCN and capture files on their own),
# smoke, the bench line, an A/B bench with the unfused heads (parity leg), rocprofv3 kernel stats.
# Stops at the first step that faults, aborts, segfaults or times out; a plain test failure
# (exit 1) is recorded and the measurement steps still run.
TAG=${1:-r3a}
O=gpurun_out/$TAG
mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "STOP after $name"; tail -30 $O/$name.log; exit $rc
  fi
  return 0
}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests 900 $PYT tests -m gpu --ignore=tests/test_gpu_capture.py --ignore=tests/test_gpu_dcn.py
grep -E "passed|failed|FAILED" $O/tests.log | tail -5
step dcn 300 $PYT tests/test_gpu_dcn.py
grep -E "passed|failed|FAILED" $O/dcn.log | tail -5
step capture 300 $PYT tests/test_gpu_capture.py
grep -E "passed|failed|FAILED|Fatal" $O/capture.log | tail -5
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
BENCH_PROFILE_OUT=$O/ops_r18.json step bench 500 python bench.py
tail -1 $O/bench.log | cut -c1-900
TV_HEADFUSE=0 step bench_nofuse 400 python bench.py --allow-env-knobs --no-b1 --no-cpu-baseline --steps 10
tail -1 $O/bench_nofuse.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('nofuse', d['value'], d.get('parity'))"
step prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o rprof --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-extras
find $O -name "*kernel_stats.csv" | head -3
