# GPU test suite against an experiment build (TV_TEST_LIB), then the per-kernel A/B of it against the
# in-tree build: bash tools/gpu_variant_tests.sh <tag> <libdir>
TAG=$1; ALT=$2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TV_TEST_LIB=tauv-vision_amd/$ALT/libtauv_vision_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests_$ALT.log 2>&1
rc=$?; echo "tests[$ALT] rc=$rc"; grep -E "passed|failed|FAILED" $O/tests_$ALT.log | tail -4
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 bash tools/gpu_libab.sh $TAG/ab lib $ALT > $O/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -14 $O/ab.log
