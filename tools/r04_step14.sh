#!/bin/bash
# round 4, step 14: graph size G for the LOCAL replay (host cost and wall
# time per iteration at S = 2 and 8, N = 4096; S = 8, N = 65536)
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r04_multishard_floor_graph_g.jsonl
: > $out
for r in 0 1; do
    timeout -k 10 120 python -u tools/r04_multishard_floor.py 1 4096 2,8 onethread >> $out || exit 1
    for G in 8 16 32 64; do
        CGX_LOCAL_GRAPH_ITERS=$G timeout -k 10 120 python -u tools/r04_multishard_floor.py 1 4096 2,8 graph >> $out || exit 1
    done
done
for G in 8 32; do
    CGX_LOCAL_GRAPH_ITERS=$G timeout -k 10 120 python -u tools/r04_multishard_floor.py 1 65536 8 graph >> $out || exit 1
done
timeout -k 10 120 python -u tools/r04_multishard_floor.py 1 65536 8 onethread >> $out || exit 1
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['n'], d['shards'], d['exchange'], d.get('graph_iters'), d['enqueue_us'], d['wall_us'], d['enqueue_10_us'], d['enqueue_16_us'])"
