# A/B a variant library against the in-tree one: parity tests on the variant, then per-op times.
#   bash tools/gpu_var_ab.sh <variant name> <op label match>
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$1; M=$2
VL=$PWD/tauv-vision_amd/lib/variants/$V.so
TV_LIB=$VL timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -k "low_precision or large_batch or u8 or determinism" > gpurun_out/var_tests.log 2>&1 && echo VAR_TESTS_OK || { echo VAR_TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/var_tests.log | head; exit 1; }
timeout -k 10 120 python tools/op_bench.py --match "$M" --tag base --reps 3 2>&1 | grep -v amdgpu.ids
TV_LIB=$VL timeout -k 10 120 python tools/op_bench.py --match "$M" --tag $V --reps 3 2>&1 | grep -v amdgpu.ids
