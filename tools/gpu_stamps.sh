#!/bin/bash
# Per-block stall/epilogue stamps of the halo convs at the bench slice size and at B=1.
set -e
mkdir -p gpurun_out/stamps
for b in 32 1; do
  TV_STAMPS=gpurun_out/stamps/b$b timeout -k 10 120 python -u tools/op_bench.py --batch $b --reps 1 --match conv --dump gpurun_out/stamps/ops$b.json > gpurun_out/stamps/op$b.log 2>&1
  python tools/stamps.py gpurun_out/stamps/b$b gpurun_out/stamps/ops$b.json > gpurun_out/stamps/sum$b.txt
done
