# GPU tests, per-kernel A/B (R18 B=32 slice) of the in-tree build against another build, then the
# B=1 per-op profile of both builds: bash tools/gpu_lat_ab.sh <tag> <libdir>
TAG=$1; ALT=$2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/tests.log | tail -4
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 bash tools/gpu_libab.sh $TAG/ab lib $ALT > $O/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -16 $O/ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
for L in lib $ALT lib $ALT; do
  TV_LIB=$GRAFT_REPO_ROOT/tauv-vision_amd/$L/libtauv_vision_amd.so timeout -k 10 120 python tools/b1_ops.py fp16 1 > $O/b1_$L.txt 2>&1; rc=$?
  echo "b1 $L rc=$rc: $(grep 'B=1' $O/b1_$L.txt) | $(grep conv_lat $O/b1_$L.txt)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
BENCH_PROFILE_OUT=$O/ops_r18.json timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; echo "bench rc=$?"
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['latency_b1'])"
