#!/bin/bash
# round 4, step 13: the LOCAL graph replay captured on one stream -- the repro
# at 2/4/8 blocks (tools/debug/graph_repro.py, with the capture traced), then
# step 12 (the bitwise tests and the host cost per iteration)
export TMPDIR=/tmp
mkdir -p gpurun_out
gcc -shared -fPIC -O1 -g -o /tmp/segv_bt.so tools/debug/segv_bt.c || exit 1
for cfg in "2 1" "4 1" "8 1" "8 8" "8 8 0"; do
    echo "== S G overlap = $cfg"
    CGX_GRAPH_DEBUG=1 timeout -k 10 60 python3 -u tools/debug/graph_repro.py $cfg > gpurun_out/r04_step13_${cfg// /_}.log 2>&1
    rc=$?
    tail -4 gpurun_out/r04_step13_${cfg// /_}.log
    [ $rc -eq 0 ] || exit $rc
done
bash tools/r04_step12.sh
