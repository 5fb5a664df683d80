# Per-op HIP-event times of one whole B=64 forward (no slicing) for R18 and DLA-34 (tools/kern_ab.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ops64
for m in r18 dla34; do
  timeout -k 10 200 python tools/kern_ab.py --model $m --batch 64 --tag $m --ops gpurun_out/ops64/ops_$m.json > gpurun_out/ops64/$m.log 2>&1; echo "$m rc=$?"
done
