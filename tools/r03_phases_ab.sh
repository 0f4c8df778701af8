#!/bin/bash
# Overhead of CGX_PHASES (in-kernel stamps) on the default bench, interleaved
# on one box: --phases off / on, two rounds.
set -u
mkdir -p gpurun_out
for round in 1 2; do
  for ph in off on; do
    timeout -k 10 240 python bench.py --phases $ph --no-cpu > gpurun_out/r03_phases_ab_${ph}_r${round}.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_phases_ab_${ph}_r${round}.json'))
p=d.get('phases_us',{}).get('per_rank',[{}])[0]
print('phases=$ph round=$round', round(d['value'],2), 'it/s', round(d['matvec_ms'],4), 'ms matvec', p)"
  done
done
