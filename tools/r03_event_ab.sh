#!/bin/bash
# A/B of the timing events' system fence (CGX_EVENT_FENCE=1 = HIP's default
# events): the default bench with the phase breakdown, interleaved.
set -u
mkdir -p gpurun_out
for round in 1 2; do
  for fence in 0 1; do
    CGX_EVENT_FENCE=$fence timeout -k 10 240 python bench.py --phases on --no-cpu --settle 3 \
        > gpurun_out/r03_event_ab_f${fence}_r${round}.json || exit $?
    python3 -c "
import json,sys;d=json.load(open('gpurun_out/r03_event_ab_f${fence}_r${round}.json'));p=d['phases_us']['per_rank'][0]
print('fence=$fence round=$round', round(d['value'],2), 'it/s', {k:p[k] for k in ('gather_exposed','combine_pap','combine_rr','gap','update_r','update_xp','iteration')})"
  done
done
