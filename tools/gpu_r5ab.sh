# conv_lat split-K thresholds at B=1: R18 and DLA-34 (hipGraph replay, fp16, 200 replays), interleaved twice
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ab; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_LAT_SPLIT=2" "TV_LAT_SPLIT_MIN=64" "TV_LAT_SPLIT_MIN=24" "TV_LAT_SPLIT=8"; do
    n=$(echo "${k:-default}" | tr ' =' '__')
    for m in r18 dla; do
      t=tools/b1_graph.py; [ $m = dla ] && t=tools/b1_dla_graph.py
      env $k timeout -k 10 120 python $t fp16 200 > $O/${m}_${rep}_$n.log 2>&1 || { echo "FAIL $m $k"; tail -3 $O/${m}_${rep}_$n.log; exit 1; }
      echo "rep $rep $m ${k:-default}: $(grep -o "'ms_per_frame': [0-9.]*" $O/${m}_${rep}_$n.log | tail -1)"
    done
  done
done
