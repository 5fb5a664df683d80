# Correctness + A/B of an alternative library build: the full GPU suite on the in-tree build,
# then the forward/parity tests with <libdir> swapped in as the in-tree library, the per-kernel
# A/B (tools/kern_ab.py) and the bench line with it. bash tools/gpu_ab_lib.sh <tag> <libdir>
TAG=$1; ALT=$2
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
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step tests 600 $PYT tests -m gpu
grep -E "passed|failed|FAILED" $O/tests.log | tail -4
L=tauv-vision_amd
mv $L/lib $L/lib_base && cp -r $L/$ALT $L/lib
step tests_alt 600 $PYT tests/test_gpu_forward.py tests/test_gpu_parity_lowp.py tests/test_gpu_dla34.py tests/test_yolact.py tests/test_gpu_backbone.py tests/test_gpu_capture.py -m gpu
grep -E "passed|failed|FAILED" $O/tests_alt.log | tail -4
step ab 300 bash tools/gpu_libab.sh $TAG/ab lib_base lib
tail -16 $O/ab.log 2>/dev/null
BENCH_PROFILE_OUT=$O/ops_alt.json step bench_alt 400 python bench.py --no-cpu-baseline --no-b1
tail -1 $O/bench_alt.log | cut -c1-700
