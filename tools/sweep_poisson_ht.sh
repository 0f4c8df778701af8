#!/bin/bash
# A/B of the halo-row load policy in the fused Poisson kernels, interleaved:
# CGX_STENCIL_HALO_T=1 (halo rows with default-policy loads) vs 0 (all nt).
set -euo pipefail
for round in 1 2; do
  for ht in 1 0; do
    for rows in ${ROWS:-8 16}; do
      out=$(CGX_STENCIL_HALO_T=$ht CGX_STENCIL_ROWS=$rows CGX_STENCIL_RB=8 timeout -k 10 120 \
            python bench.py --workload poisson --no-cpu --steps 20 --warmup 3)
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $round, 'halo_t': $ht, \
'rows': $rows, 'it_s': d['value'], 'xr_ms': d['matvec_ms'], 'iter_gbps': d['iteration_gbps']}))" "$out"
    done
  done
done
