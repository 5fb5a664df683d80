set -e
O=gpurun_out/dbg; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/dbg_lowp.py dla34 b1_480x640_kp fp16 64 > $O/on.log 2>&1 && echo ON_OK
TV_LAT=0 timeout -k 10 200 python tools/dbg_lowp.py dla34 b1_480x640_kp fp16 64 > $O/off.log 2>&1 && echo OFF_OK
cat $O/on.log | tail -20; echo ----; cat $O/off.log | tail -20
