# conv3x3 half-tile cost knob sweep (R18 B=64 + B=1, DLA-34, YOLACT); default is 55
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ag; mkdir -p $O
v() { tail -1 $1 | grep -o '"value": [0-9.]*'; }
for rep in 1 2; do
  for c in 55 62 70 85 100; do
    TV_C3_HALF_COST=$c timeout -k 10 300 python bench.py --allow-env-knobs --no-cpu-baseline --no-extras --steps 20 > $O/r18_${rep}_$c.log 2>&1 || { echo "FAIL r18 $c"; exit 1; }
    echo "rep $rep r18 cost $c: $(v $O/r18_${rep}_$c.log) b1 $(tail -1 $O/r18_${rep}_$c.log | grep -o '"ms_per_frame": [0-9.]*' | head -1)"
  done
done
for m in dla34 yolact; do
  for c in 55 70 100; do
    TV_C3_HALF_COST=$c timeout -k 10 300 python bench.py --model $m --allow-env-knobs --no-cpu-baseline --no-extras --steps 20 > $O/${m}_$c.log 2>&1 || { echo "FAIL $m $c"; exit 1; }
    echo "$m cost $c: $(v $O/${m}_$c.log) b1 $(tail -1 $O/${m}_$c.log | grep -o '"ms_per_frame": [0-9.]*' | head -1)"
  done
done
