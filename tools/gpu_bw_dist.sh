# HBM stream ceilings (tools/micro: write-only / read-only / read+write, the stem's and ConvT's
# shapes), then the multi-rank bench path under torch.distributed.run with RCCL at N=1:
# bash tools/gpu_bw_dist.sh <tag>
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 tools/micro/wr_pattern > $O/wr_pattern.txt 2>&1; rc=$?; echo "wr rc=$rc"; cat $O/wr_pattern.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 tools/micro/rw_pattern > $O/rw_pattern.txt 2>&1; rc=$?; echo "rw rc=$rc"; cat $O/rw_pattern.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_dist1.log 2>&1; rc=$?; echo "dist bench rc=$rc"
tail -1 $O/bench_dist1.log | cut -c1-600
