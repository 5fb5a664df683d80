TAG=r3b
O=gpurun_out/$TAG
mkdir -p $O
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
grep -E "passed|failed|FAILED" $O/tests.log | tail -4
BENCH_PROFILE_OUT=$O/ops_r18.json step bench 400 python bench.py --no-cpu-baseline --no-b1
tail -1 $O/bench.log | cut -c1-900
for L in lib_s9 lib_s9b; do
  TV_LIB=$GRAFT_REPO_ROOT/tauv-vision_amd/$L/libtauv_vision_amd.so step st_$L 200 python tools/c3_stamps.py --match ida_up_reverse.output_layers.0.0
  tail -14 $O/st_$L.log
done
