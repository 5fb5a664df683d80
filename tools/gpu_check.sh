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
step tests 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -6
BENCH_PROFILE_OUT=$O/ops_r18.json step bench_r18 500 python bench.py ${BENCH_ARGS:-}
tail -1 $O/bench_r18.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r18', d['value'], d['ms_per_step'], d.get('launch'), 'eager', d.get('eager_value'), 'frac', d['roofline']['frac'], 'e2e', d['e2e_frac_of_peak'], 'parity', d.get('parity', {}).get('max_box_err'))"
for m in dla34 yolact; do
  BENCH_PROFILE_OUT=$O/ops_$m.json step bench_$m 300 python bench.py --model $m --no-cpu-baseline --no-extras --no-b1
  tail -1 $O/bench_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d.get('launch'), 'eager', d.get('eager_value'), 'frac', d['roofline']['frac'], d.get('mask_roofline', {}).get('achieved'))"
done
