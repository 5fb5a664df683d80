#!/bin/bash
# parity tests (forward subset) against each named variant library, then tools/gpu_abl.sh timings
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for v in "$@"; do
  TV_LIB=$PWD/tauv-vision_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -k "low_precision or large_batch or u8 or batched" > gpurun_out/abl/t_$v.log 2>&1 && echo "$v TESTS_OK" || { echo "$v TESTS_FAIL"; grep -E "FAILED|Error" gpurun_out/abl/t_$v.log | head -3; }
done
bash tools/gpu_abl.sh "$@"
