#!/bin/bash
# Timing-only ablations of the 3x3 halo conv (tools/variants/c3_abl.hip): per-op times at B=32
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for v in "$@"; do
  TV_LIB=$PWD/tauv-vision_amd/lib/variants/$v.so timeout -k 10 120 python tools/op_bench.py --batch 32 --reps 3 --tag $v > gpurun_out/abl/$v.log 2>&1
  grep total gpurun_out/abl/$v.log
done
