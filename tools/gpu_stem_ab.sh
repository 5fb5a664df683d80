set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "u8 or low_precision or large_batch or determinism" > gpurun_out/stem_tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/stem_tests.log | head; exit 1; }
for a in ${ABL:-0 1 2 4 6}; do
  TV_STEM_ABLATE=$a timeout -k 10 120 python tools/op_bench.py --match dla_down.projection_layer --tag abl$a --reps 3 2>&1 | grep -v total
done
