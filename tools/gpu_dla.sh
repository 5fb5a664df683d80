#!/bin/bash
# full GPU test suite, then DLA34 bench (+ per-launch profile) and the R18 headline bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dla
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dla/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/dla/tests.log; exit 1; }
tail -2 gpurun_out/dla/tests.log
TV_PROFILE_OUT=gpurun_out/dla/ops_dla34_b64.json timeout -k 10 300 python bench.py --model dla34 --steps 10 --warmup 3 --cpu-seconds 15 > gpurun_out/dla/bench_dla34.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/dla/bench_dla34.log; exit 1; }
tail -1 gpurun_out/dla/bench_dla34.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dla/bench_r18.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/dla/bench_r18.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/dla/bench_r18.log').read().strip().splitlines()[-1]); print('R18', d['value'], 'fps', d['latency_b1']['ms_per_frame'], 'ms B=1')"
