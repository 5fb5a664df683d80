cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slices
for sl in 2 1 3 4 2; do
  TV_SLICES=$sl timeout -k 10 200 python bench.py --allow-env-knobs --no-extras --no-cpu-baseline --no-b1 > gpurun_out/slices/s$sl.log 2>&1; echo "slices=$sl rc=$?"
  tail -1 gpurun_out/slices/s$sl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('  value', d['value'], 'ms', d['ms_per_step'])"
done
