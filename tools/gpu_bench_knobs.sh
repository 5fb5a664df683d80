# Whole-step bench A/B of engine knob settings, interleaved twice (box drift), with the B=1
# latency leg: bash tools/gpu_bench_knobs.sh <tag> default "TV_SLICE_SIZES=40,24" ... (BENCH_ARGS="--model dla34" for another model)
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  i=0
  for K in "$@"; do
    i=$((i + 1))
    if [ "$K" = default ]; then
      timeout -k 10 300 python bench.py $BENCH_ARGS --no-cpu-baseline --no-extras --steps 30 > $O/b_$i.$rep.log 2>&1 || exit $?
    else
      env $K timeout -k 10 300 python bench.py $BENCH_ARGS --allow-env-knobs --no-cpu-baseline --no-extras --steps 30 > $O/b_$i.$rep.log 2>&1 || exit $?
    fi
    python -c "import json; d=json.loads(open('$O/b_$i.$rep.log').read().strip().splitlines()[-1]); b=d.get('latency_b1') or {}; print('$K', $rep, d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in b.items()})"
  done
done
