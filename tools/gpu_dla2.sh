#!/bin/bash
# DLA34 tests + DLA34 bench with per-launch profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dla
timeout -k 10 300 python -u -m pytest tests/test_gpu_dla34.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dla/tests2.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/dla/tests2.log; exit 1; }
tail -1 gpurun_out/dla/tests2.log
TV_PROFILE_OUT=gpurun_out/dla/ops_dla34_b64.json timeout -k 10 300 python bench.py --model dla34 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dla/bench_dla34.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/dla/bench_dla34.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/dla/bench_dla34.log').read().strip().splitlines()[-1]); print('DLA34', d['value'], 'fps', d['latency_b1']['ms_per_frame'], 'ms B=1')"
