# GPU tests on the in-tree build, then the per-kernel A/B of the in-tree build against another
# build (tools/gpu_libab.sh), then the bench line: bash tools/gpu_libab2.sh <tag> <libdir>
TAG=$1; ALT=$2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/tests.log | tail -4
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 300 bash tools/gpu_libab.sh $TAG/ab lib $ALT > $O/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -16 $O/ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_PROFILE_OUT=$O/ops_r18.json timeout -k 10 400 python bench.py --model ${MODEL:-r18} --no-cpu-baseline --no-b1 > $O/bench.log 2>&1; echo "bench rc=$?"
tail -1 $O/bench.log | cut -c1-700
