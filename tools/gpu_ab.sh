# A/B of engine env switches on per-op times: bash tools/gpu_ab.sh <match> "<ENV=.. ENV=..>" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
M=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/ab_tests.log | head; exit 1; }
for v in "$@"; do
  env $v timeout -k 10 120 python tools/op_bench.py --match "$M" --tag "[$v]" --reps 3 2>&1 | grep -v amdgpu.ids
done
