#!/bin/bash
# CGX_SYMMETRIC at N=65536: blocks per CU (1 / 2) and tile-load policy, interleaved
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "2 1" "1 1" "2 0"; do
    set -- $cfg
    CGX_SYM_BLOCKS_PER_CU=$1 CGX_SYM_NT=$2 timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 50 \
        > gpurun_out/r03_symab_b$1_nt$2_r$r.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_symab_b$1_nt$2_r$r.json'))
print('blocks/CU=$1 nt=$2 round=$r', round(d['value'],1), 'it/s', round(d['roofline']['achieved'],1), 'GB/s')"
  done
done
