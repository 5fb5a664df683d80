# R18 B=64 slice-schedule knob sweep at the half-tile cost 70 default (2 reps, one box)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ai; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_SLICES=3" "TV_SLICES=4" "TV_SLICE_SIZES=28,36" "TV_SLICE_SIZES=24,40" "TV_SLICE_LAG=3" "TV_HALF=x"; do
    n=$(echo "${k:-default}" | tr ' =,' '___')
    [ "$k" = "TV_HALF=x" ] && k="TV_C3_HALF_COST=85 TV_SLICE_SIZES=36,28"
    env $k timeout -k 10 300 python bench.py --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 20 > $O/k_${rep}_$n.log 2>&1 || { echo "FAIL $k"; exit 1; }
    echo "rep $rep ${k:-default}: $(tail -1 $O/k_${rep}_$n.log | grep -o '"value": [0-9.]*')"
  done
done
