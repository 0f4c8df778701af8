#!/bin/bash
# round 4, step 19: the Poisson plan knobs re-checked on the final tree
# (XCD bands, the reverse walk of the xr kernels, rows per step of the plain
# kernels), interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_variants.py --rounds 3 --args "--workload poisson --steps 300" \
    --variant default= --variant bands0=CGX_POISSON_BANDS=0 --variant rev0=CGX_STENCIL_REVERSE=0 \
    --variant rb4=CGX_STENCIL_RB=4 \
    > gpurun_out/r04_poisson_knobs_ab.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r04_poisson_knobs_ab.jsonl'):
    d=json.loads(l); print(d.get('variant'), d.get('round'), d.get('value'))"
