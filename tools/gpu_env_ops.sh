#!/bin/bash
# per-op times (tools/op_bench.py) under engine env switches: bash tools/gpu_env_ops.sh <batch> "<tag>:<ENV=..>" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
b=$1; shift
for tv in "$@"; do
  t=${tv%%:*}; v=${tv#*:}
  env $v timeout -k 10 120 python tools/op_bench.py --batch $b --reps 3 --tag $t > gpurun_out/abl/$t.log 2>&1
  grep total gpurun_out/abl/$t.log
done
