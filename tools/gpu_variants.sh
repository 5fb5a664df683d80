# A/B the library variants under tauv-vision_amd/lib/variants (bench + per-kernel op times)
set -e
mkdir -p gpurun_out/var
for v in "$@"; do
  TV_LIB=$PWD/tauv-vision_amd/lib/variants/$v.so TV_PROFILE_OUT=gpurun_out/var/ops_$v.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b1 > gpurun_out/var/b_$v.log 2>&1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
line = json.loads(open(f"gpurun_out/var/b_{v}.log").read().strip().splitlines()[-1])
ops = json.load(open(f"gpurun_out/var/ops_{v}.json"))
agg = {}
for o in ops:
    k = o["kernel"].split("<")[0]
    a = agg.setdefault(k, [0.0, 0.0])
    a[0] += o["ms"]; a[1] += o["gflop"]
print(v, "fps", line["value"], " ".join(f"{k}:{a[0]:.3f}ms/{a[1]/max(a[0],1e-9):.0f}TF" for k, a in agg.items()))
PY
done
