# Quick iteration call: GPU tests (or a subset: $2 = pytest -k expr), bench line + per-op times.
set -e
TAG=${1:-q}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
K=${2:-}
if [ -n "$K" ]; then KA="-k $K"; else KA=""; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread $KA > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
TV_PROFILE_OUT=$O/ops.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-400
python tools/opsum.py $O/ops.json
