#!/bin/bash
# CGX_SYMMETRIC: one or two 256-thread blocks per CU at N = 65536 / 16384,
# interleaved (odd units per block in both), on whatever box this lands.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 65536 16384; do
  for r in 1 2; do
    for b in 1 2 1 2; do
      CGX_SYM_BLOCKS_PER_CU=$b timeout -k 10 240 python bench.py --workload symmetric --n $n --no-cpu --steps 50 \
          > gpurun_out/r03_symbpc.json || exit $?
      python3 -c "
import json;d=json.load(open('gpurun_out/r03_symbpc.json'))
print(json.dumps({'n': $n, 'blocks_per_cu': $b, 'it_s': round(d['value'],1), 'gbps': round(d['roofline']['achieved'],1)}))" | tee -a gpurun_out/r03_sym_bpc_ab.jsonl
    done
  done
done
