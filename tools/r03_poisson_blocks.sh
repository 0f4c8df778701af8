#!/bin/bash
# Poisson configs[4]: resident blocks of the fused kernels (CGX_STENCIL_BLOCKS;
# default = occupancy x CUs: 4 / CU for k_poisson_p, 3 / CU for k_poisson_xr)
# against 2 and 3 per CU for both, interleaved.
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_pblocks
mkdir -p $D
for r in 1 2; do
  for b in default 512 768; do
    if [ $b = default ]; then unset CGX_STENCIL_BLOCKS; else export CGX_STENCIL_BLOCKS=$b; fi
    timeout -k 10 200 python bench.py --workload poisson --no-cpu --steps 200 > $D/b${b}_r$r.json 2>/dev/null || exit $?
    python3 -c "
import json;d=json.load(open('$D/b${b}_r$r.json'));print('blocks=$b r$r', round(d['value'],1),'it/s')"
  done
done
