#!/bin/bash
# DLA34 + R18 measurement evidence: full bench lines (with CPU baseline) and rocprofv3 kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
mkdir -p gpurun_out/r1d
TV_PROFILE_OUT=gpurun_out/r1d/ops_dla34_b64_fp16.json timeout -k 10 300 python bench.py --model dla34 --cpu-seconds 15 > gpurun_out/r1d/bench_dla34.log 2>&1 || { echo BENCH_FAIL; tail gpurun_out/r1d/bench_dla34.log; exit 1; }
tail -1 gpurun_out/r1d/bench_dla34.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1d/prof -o dla34 --output-format csv -- python bench.py --model dla34 --steps 10 --warmup 3 --no-cpu-baseline --no-b1 > gpurun_out/r1d/prof_dla34.log 2>&1 || { echo PROF_FAIL; tail gpurun_out/r1d/prof_dla34.log; exit 1; }
TV_PROFILE_OUT=gpurun_out/r1d/ops_r18_b64_fp16.json timeout -k 10 300 python bench.py > gpurun_out/r1d/bench_r18.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/r1d/bench_r18.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1d/prof -o r18 --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b1 > gpurun_out/r1d/prof_r18.log 2>&1 || { echo PROF_FAIL; exit 1; }
find gpurun_out/r1d -name "*stats*"
