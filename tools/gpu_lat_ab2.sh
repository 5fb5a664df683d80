# tools/gpu_lat_ab.sh (tests, R18 per-kernel A/B, B=1 per-op, bench line), then the DLA-34
# per-kernel A/B: bash tools/gpu_lat_ab2.sh <tag> <libdir>
TAG=$1; ALT=$2
bash tools/gpu_lat_ab.sh $TAG $ALT || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MODEL=dla34 timeout -k 10 300 bash tools/gpu_libab.sh $TAG/ab_dla34 lib $ALT > gpurun_out/$TAG/ab_dla34.log 2>&1; rc=$?; echo "ab dla34 rc=$rc"; tail -16 gpurun_out/$TAG/ab_dla34.log
