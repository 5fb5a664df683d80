# A/B a variant library: parity tests on it, then op totals at B=64 and B=1 for base and variant
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$1
VL=$PWD/tauv-vision_amd/lib/variants/$V.so
TV_LIB=$VL timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -k "low_precision or large_batch or u8 or determinism or batched" > gpurun_out/var_tests.log 2>&1 && echo VAR_TESTS_OK || { echo VAR_TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/var_tests.log | head; exit 1; }
for b in 64 1; do
  timeout -k 10 120 python tools/op_bench.py --batch $b --match "@@" --tag "base B=$b" --reps 3 2>&1 | grep total
  TV_LIB=$VL timeout -k 10 120 python tools/op_bench.py --batch $b --match "@@" --tag "$V B=$b" --reps 3 2>&1 | grep total
done
