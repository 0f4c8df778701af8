#!/bin/bash
# Fused Poisson kernel plan sweep (run on the GPU box from the repo root):
# rows per step RB x rows per work item x grid blocks; one bench run per point.
#   ROWS="8 16" RBS="4 8" BLOCKS="0 2048" bash tools/sweep_poisson.sh > gpurun_out/sweep_poisson.jsonl
# BLOCKS 0 = the occupancy-sized default.
set -euo pipefail
for blocks in ${BLOCKS:-0}; do
  for rows in ${ROWS:-8 16 32}; do
    for rb in ${RBS:-2 4 8}; do
      if [ "$blocks" = 0 ]; then unset CGX_STENCIL_BLOCKS; else export CGX_STENCIL_BLOCKS=$blocks; fi
      out=$(CGX_STENCIL_ROWS=$rows CGX_STENCIL_RB=$rb timeout -k 10 120 \
            python bench.py --workload poisson --no-cpu --steps 20 --warmup 3)
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'blocks': $blocks, 'rows': $rows, \
'rb': $rb, 'it_s': d['value'], 'xr_ms': d['matvec_ms'], 'xr_gbps': d['roofline']['achieved'], \
'iter_gbps': d['iteration_gbps']}))" "$out"
    done
  done
done
