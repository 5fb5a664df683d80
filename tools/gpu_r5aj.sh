# DLA-34 B=64 knob sweep (2 reps, one box)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5aj; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_C3_HALF_COST=85" "TV_C3_HALF_COST=0" "TV_SLICES=1" "TV_SLICES=3" "TV_DCN64=0" "TV_C1X1=2" "TV_LAT_UNITS=128" "TV_LAT_UNITS=512"; do
    n=$(echo "${k:-default}" | tr ' =,' '___')
    env $k timeout -k 10 300 python bench.py --model dla34 --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 20 > $O/k_${rep}_$n.log 2>&1 || { echo "FAIL $k"; exit 1; }
    echo "rep $rep ${k:-default}: $(tail -1 $O/k_${rep}_$n.log | grep -o '"value": [0-9.]*')"
  done
done
