# bench.py fps under engine env switches: bash tools/gpu_env_bench.sh "<ENV=..>" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-b1 > gpurun_out/envb.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/envb.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], 'fps', d['ms_per_step'], 'ms')"
done
