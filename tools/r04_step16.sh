#!/bin/bash
# round 4, step 16: Poisson items of 16 rows (half the halo-row re-reads)
# against the default 8, interleaved; the pipelined catch-up needs 8-row
# items, so "r8plain" is the default with it off (the fair 8-vs-16 pair)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_variants.py --rounds 3 --args "--workload poisson --steps 300" \
    --variant default= --variant r8plain=CGX_XR_PIPE_CATCHUP=0 --variant r16=CGX_STENCIL_ROWS=16 \
    --variant r12=CGX_STENCIL_ROWS=12 \
    > gpurun_out/r04_poisson_rows_ab.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r04_poisson_rows_ab.jsonl'):
    d=json.loads(l); print(d.get('variant'), d.get('round'), d.get('value'))"
