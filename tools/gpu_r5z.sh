# B=1 latency knob A/B round 2 (R18 fp16 + DLA-34 fp16) and the B=64 line with conv_lat split-K off
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5z; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_LAT_SPLIT=1" "TV_LAT_SPLIT=2" "TV_LAT_SPLIT=1 TV_LATGROUP=0" "TV_LAT_SPLIT=1 TV_LAT_UNITS=128" "TV_LAT_SPLIT=1 TV_LAT_UNITS=512"; do
    n=$(echo "${k:-default}" | tr ' =' '__')
    env $k timeout -k 10 120 python tools/b1_graph.py fp16 200 > $O/b1_${rep}_$n.log 2>&1 || { echo "FAIL $k"; tail -3 $O/b1_${rep}_$n.log; exit 1; }
    echo "rep $rep ${k:-default}: $(grep -o "'ms_per_frame': [0-9.]*" $O/b1_${rep}_$n.log | tail -1)"
  done
done
for k in "" "TV_LAT_SPLIT=1"; do
  n=$(echo "${k:-default}" | tr ' =' '__')
  env $k timeout -k 10 300 python bench.py --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 30 > $O/bench_$n.log 2>&1 || { echo "FAIL bench $k"; exit 1; }
  echo "B=64 ${k:-default}: $(tail -1 $O/bench_$n.log | grep -o '"value": [0-9.]*')"
  env $k timeout -k 10 300 python bench.py --model dla34 --allow-env-knobs --no-cpu-baseline --no-extras --steps 20 > $O/dla_$n.log 2>&1 || { echo "FAIL dla $k"; exit 1; }
  echo "DLA ${k:-default}: $(tail -1 $O/dla_$n.log | grep -o '"value": [0-9.]*') $(tail -1 $O/dla_$n.log | grep -o '"fp16": {[^}]*}' | grep -o 'ms_per_frame": [0-9.]*')"
done
