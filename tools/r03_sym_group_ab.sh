#!/bin/bash
# CGX_SYMMETRIC at N=65536: column-partial barrier per unit (0), per pair (1),
# per group of four units (2), interleaved; the symmetric tests first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_symmetric.py -q --timeout 300 --timeout-method thread -m gpu \
    -p no:cacheprovider > gpurun_out/r03_sym_group_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_sym_group_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1 2; do
    CGX_SYM_PAIR=$v timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 50 \
        > gpurun_out/r03_symgrp${v}_r$r.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_symgrp${v}_r$r.json'))
print(json.dumps({'group': $v, 'n': 65536, 'round': $r, 'it_s': round(d['value'],1), 'gbps': round(d['roofline']['achieved'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_sym_group_ab.jsonl
  done
done
