#!/bin/bash
# Interleaved A/B of one environment knob on a bench workload (GPU box, repo root):
#   VAR=CGX_POISSON_PLAN VALUES="reverse=0 reverse=1" ROUNDS=3 ARGS="--workload poisson" bash tools/ab_env.sh
set -euo pipefail
for round in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VALUES:-0 1}; do
    out=$(env "$VAR=$v" timeout -k 10 150 python bench.py --no-cpu ${ARGS:-})
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $round, '$VAR': '$v', \
'value': d['value'], 'kernel_ms': d['matvec_ms'], 'kernel_gbps': d['roofline']['achieved'], \
'iteration_gbps': d.get('iteration_gbps')}))" "$out"
  done
done
