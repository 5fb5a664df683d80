# YOLACT bench line of the in-tree build vs another build, interleaved twice:
# bash tools/gpu_yolact_ab.sh <tag> <libdir>
TAG=$1; ALT=$2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for L in lib $ALT; do
    TV_LIB=$GRAFT_REPO_ROOT/tauv-vision_amd/$L/libtauv_vision_amd.so BENCH_PROFILE_OUT=$O/ops_yolact_$L.$rep.json timeout -k 10 300 python bench.py --model yolact --no-cpu-baseline --allow-env-knobs > $O/bench_$L.$rep.log 2>&1; rc=$?
    echo "$L.$rep rc=$rc $(tail -1 $O/bench_$L.$rep.log | cut -c1-140)"
    if [ $rc -ne 0 ]; then tail -5 $O/bench_$L.$rep.log; exit $rc; fi
  done
done
