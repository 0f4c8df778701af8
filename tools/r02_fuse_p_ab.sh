#!/bin/bash
# Two-launch dense iteration (CGX_FUSE_P=1: the x/r update's last block forms p
# for the whole vector) against three launches above its default n <= 8192,
# interleaved bench runs (fixed-count iterations, no CPU leg).
set -euo pipefail
OUT=gpurun_out/fuse_p_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
    for n in 12288 16384 24576; do
        for f in 0 1; do
            CGX_FUSE_P=$f timeout -k 10 120 python bench.py --n $n --steps 300 --warmup 20 --settle 1 --no-cpu \
                | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({'n': $n, 'CGX_FUSE_P': $f, 'it_s': d['value'], 'ms_per_step': d['ms_per_step'], 'matvec_ms': d['matvec_ms'], 'relres': d['check']['relres']}))" >> $OUT
        done
    done
done
cat $OUT
