#!/bin/bash
# Fused Poisson kernel plan sweep (run on the GPU box from the repo root):
# (rows per work item, rows per step RB) pairs x grid blocks, interleaved rounds.
#   PAIRS="8:8 4:4" BLOCKS="0 2048" ROUNDS=2 bash tools/sweep_poisson.sh > gpurun_out/sweep_poisson.jsonl
# BLOCKS 0 = the occupancy-sized default.
set -euo pipefail
for round in $(seq 1 ${ROUNDS:-1}); do
  for blocks in ${BLOCKS:-0}; do
    for pair in ${PAIRS:-8:8 16:8 8:4 4:4}; do
      rows=${pair%:*}; rb=${pair#*:}
      if [ "$blocks" = 0 ]; then unset CGX_STENCIL_BLOCKS; else export CGX_STENCIL_BLOCKS=$blocks; fi
      out=$(CGX_STENCIL_ROWS=$rows CGX_STENCIL_RB=$rb timeout -k 10 120 \
            python bench.py --workload poisson --no-cpu --steps 20 --warmup 3)
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $round, 'blocks': $blocks, \
'rows': $rows, 'rb': $rb, 'it_s': d['value'], 'xr_ms': d['matvec_ms'], 'xr_gbps': d['roofline']['achieved'], \
'iter_gbps': d['iteration_gbps']}))" "$out"
    done
  done
done
