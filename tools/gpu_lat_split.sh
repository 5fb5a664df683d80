# B=1 per-op latency (tools/b1_ops.py) at conv_lat split-K factors 1, 2, 4, 8 (knob TV_LAT_SPLIT),
# twice each: bash tools/gpu_lat_split.sh <tag>
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for k in 1 2 4 8; do
    TV_LAT_SPLIT=$k timeout -k 10 120 python tools/b1_ops.py fp16 1 > $O/b1_split$k.$rep.txt 2>&1; rc=$?
    echo "split $k rep $rep rc=$rc: $(grep 'B=1' $O/b1_split$k.$rep.txt) | $(grep conv_lat $O/b1_split$k.$rep.txt)"
    if [ $rc -ne 0 ]; then tail -5 $O/b1_split$k.$rep.txt; exit $rc; fi
  done
done
