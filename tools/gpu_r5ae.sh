# convt3 forced tile shapes (tools/ct3_time.py: both protonet layers at B=32), kernel trace per shape
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ae; mkdir -p $O
for t in "0 0" "16 16" "23 11" "18 14" "32 8" "12 21" "28 9" "8 32"; do
  n=$(echo $t | tr ' ' 'x')
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$n -o run -- python tools/ct3_time.py tauv-vision_amd/lib/libtauv_vision_amd.so $t > $O/$n.log 2>&1 || { echo "fail $n"; tail -3 $O/$n.log; exit 1; }
done
echo done
