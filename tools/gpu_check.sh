# Quick check of a change: all GPU tests, then the bench lines (R18 default incl. extras; DLA-34 and
# YOLACT without CPU baseline / extras / B=1) with per-op HIP-event times. Outputs under
# gpurun_out/<tag>/. Stops at the first step that faults, aborts, segfaults or times out.
TAG=${1:-chk}
O=gpurun_out/$TAG
mkdir -p $O
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
step tests 900 python -u -m pytest --maxfail=${MAXFAIL:-1} -v --timeout 120 --timeout-method thread ${TESTS:-tests} -m gpu
grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -6
BENCH_PROFILE_OUT=$O/ops_r18.json step bench_r18 500 python bench.py ${BENCH_ARGS:-}
tail -1 $O/bench_r18.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r18', d['value'], d['ms_per_step'], d.get('launch'), 'eager', d.get('eager_value'), 'frac', d['roofline']['frac'], d['roofline'].get('frac_best'), 'e2e', d['e2e_frac_of_peak'], 'api', d.get('api'), 'node', d.get('node_b1'), 'b1', {k: v['ms_per_frame'] for k, v in (d.get('latency_b1') or {}).items()})"
for m in ${MODELS-dla34 yolact}; do
  BENCH_PROFILE_OUT=$O/ops_$m.json step bench_$m 300 python bench.py --model $m --no-cpu-baseline --no-extras --no-b1
  tail -1 $O/bench_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d.get('launch'), 'eager', d.get('eager_value'), 'frac', d['roofline']['frac'], d.get('mask_roofline', {}).get('achieved'))"
done
# optional: TIMELINE=1 -> kernel trace of a short bench run + tools/timeline.py (per-family wall time)
if [ -n "${TIMELINE:-}" ]; then
  step trace 300 rocprofv3 --kernel-trace -d $O/prof -o trace --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-b1 --no-extras
  python tools/timeline.py "$(find $O/prof -name '*kernel_trace.csv' | head -1)" > $O/timeline.txt 2>&1; cat $O/timeline.txt
fi
# optional: MICRO=1 -> FETCH_SIZE calibration of the halo read pattern (tools/micro/halo_fetch.hip, prebuilt)
if [ -n "${MICRO:-}" ]; then
  step micro 60 tools/micro/halo_fetch
  cat $O/micro.log
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_micro -o fetch --output-format csv -- tools/micro/halo_fetch > $O/micro_pmc.log 2>&1; echo "micro pmc rc=$?"
fi
