# tests, then bench fps of the in-tree library vs a reference build (lib/variants/<name>.so, first argument)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abold_tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/abold_tests.log | head; exit 1; }
for i in 1 2; do
for v in "" "$PWD/tauv-vision_amd/lib/variants/${1:-base}.so"; do
  TV_LIB=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-b1 > gpurun_out/envb.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/envb.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], 'fps')"
done
done
