#!/bin/bash
# Poisson m=8192: each XCD band's walk rotated by x * ROT items
# (CGX_POISSON_BAND_ROT = 0 / 1 / 17 / 129), bench processes interleaved; the
# Poisson tests under ROT=17 first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
CGX_POISSON_BAND_ROT=17 timeout -k 10 600 python -u -m pytest tests -q --timeout 500 --timeout-method thread -m gpu \
    -k poisson -p no:cacheprovider > gpurun_out/r03_poisson_rot_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_poisson_rot_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for rot in 0 1 17 129; do
    CGX_POISSON_BAND_ROT=$rot timeout -k 10 240 python bench.py --workload poisson --no-cpu --steps 200 \
        > gpurun_out/r03_prot.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_prot.json'))
print(json.dumps({'rot': $rot, 'round': $r, 'it_s': round(d['value'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_poisson_rot_ab.jsonl
  done
done
