#!/bin/bash
# split-K A/B: GPU tests, per-op totals at B=1 and B=32, bench (B=64 + B=1 latency)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sk_tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/sk_tests.log | head; exit 1; }
bash tools/gpu_env_ops.sh 1 sk0:TV_C3_SK=0 sk1:TV_C3_SK=1
bash tools/gpu_env_ops.sh 32 sk0b32:TV_C3_SK=0 sk1b32:TV_C3_SK=1
for v in TV_C3_SK=0 TV_C3_SK=1; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/envb.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/envb.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], 'fps', d['latency_b1']['ms_per_frame'], 'ms B=1')"
done
