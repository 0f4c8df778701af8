#!/bin/bash
# round 4, step 12: the one-process multi-shard loop replayed from hipGraphs
# (CGX_LOCAL_GRAPH): the bitwise tests, then the host cost per iteration
# against the eager one-thread enqueue at S = 2/4/8 (G = 8 and 32)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -m gpu -q --timeout 200 --timeout-method thread \
    -k "local_graph or local_exchange" > gpurun_out/r04_step12_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_step12_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r04_multishard_floor.py 2 4096 2,4,8 onethread,graph > gpurun_out/r04_multishard_floor_graph.jsonl || exit 1
CGX_LOCAL_GRAPH_ITERS=32 timeout -k 10 300 python -u tools/r04_multishard_floor.py 1 4096 8 graph >> gpurun_out/r04_multishard_floor_graph.jsonl || exit 1
timeout -k 10 300 python -u tools/r04_multishard_floor.py 1 65536 8 onethread,graph >> gpurun_out/r04_multishard_floor_graph.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r04_multishard_floor_graph.jsonl'):
    d=json.loads(l); print(d['n'], d['shards'], d['exchange'], d.get('graph_iters'), d['enqueue_us'], d['wall_us'], d['enqueue_10_us'], d['enqueue_16_us'])"
