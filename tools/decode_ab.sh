cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dec
for v in base nosel_tile nosel_both; do
  if [ $v = base ]; then L=""; else L="TV_LIB=$GRAFT_REPO_ROOT/tauv-vision_amd/lib/variants/$v.so"; fi
  env $L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/dec/p_$v -o p --output-format csv -- python tools/decode_bench.py --only > gpurun_out/dec/$v.log 2>&1 || exit 1
  echo "== $v"; grep -E "select" gpurun_out/dec/p_$v/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-30,100-200
done
