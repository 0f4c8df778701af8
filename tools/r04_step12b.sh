#!/bin/bash
# round 4, step 12b: step 12's host-cost measurements alone (after its tests passed)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r04_multishard_floor.py 2 4096 2,4,8 onethread,graph > gpurun_out/r04_multishard_floor_graph.jsonl || exit 1
CGX_LOCAL_GRAPH_ITERS=32 timeout -k 10 300 python -u tools/r04_multishard_floor.py 1 4096 8 graph >> gpurun_out/r04_multishard_floor_graph.jsonl || exit 1
timeout -k 10 300 python -u tools/r04_multishard_floor.py 1 65536 8 onethread,graph >> gpurun_out/r04_multishard_floor_graph.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r04_multishard_floor_graph.jsonl'):
    d=json.loads(l); print(d['n'], d['shards'], d['exchange'], d.get('graph_iters'), d['enqueue_us'], d['wall_us'], d['enqueue_10_us'], d['enqueue_16_us'])"
