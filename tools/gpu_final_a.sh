# Round measurement, part 1 (tests, smoke, bench lines): GPU tests + smoke, the R18 bench line (defaults: CPU baseline, B=1 latency,
# extras), DLA-34 and YOLACT lines, rocprofv3 kernel stats of each, PMC FETCH/WRITE passes (R18 and
# DLA-34 forwards) and the MFMA-utilisation pass. Outputs under gpurun_out/<tag>/. Stops at the
# first step that faults, aborts, segfaults or times out.
TAG=${1:-r3}
O=gpurun_out/$TAG
mkdir -p $O/prof $O/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; tail -30 $O/$name.log; exit $rc; fi
  return 0
}
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
grep -E "passed|failed|FAILED" $O/tests.log | tail -3
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
BENCH_PROFILE_OUT=$O/ops_r18.json step bench_r18 500 python bench.py
tail -1 $O/bench_r18.log | cut -c1-400
for m in dla34 yolact; do
  BENCH_PROFILE_OUT=$O/ops_$m.json step bench_$m 300 python bench.py --model $m --cpu-seconds 10
  tail -1 $O/bench_$m.log | cut -c1-300
done
