# B=1 latency knob A/B (hipGraph replay, R18 fp16, 200 replays each, interleaved twice)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5y; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_STEMFUSE=0" "TV_BURST=0" "TV_LAT_SPLIT=1" "TV_C3_NW=8"; do
    env $k timeout -k 10 120 python tools/b1_graph.py fp16 200 > $O/b1_${rep}_${k:-default}.log 2>&1 || { echo "FAIL $k"; tail -3 $O/b1_${rep}_${k:-default}.log; exit 1; }
    echo "rep $rep ${k:-default}: $(grep ms_per_frame $O/b1_${rep}_${k:-default}.log | tail -1)"
  done
done
