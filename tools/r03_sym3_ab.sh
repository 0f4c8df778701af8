#!/bin/bash
# k_symv3_f64 (three slots, CGX_SYM_SLOTS=3) against the two-slot kernel:
# the symmetric tests with three slots, then bench lines interleaved.
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_sym3
mkdir -p $D
CGX_SYM_SLOTS=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_symmetric.py -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1
rc=$?
tail -2 $D/tests.log
[ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  for sl in 2 3; do
    CGX_SYM_SLOTS=$sl timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/s${sl}_r$r.json 2>/dev/null || exit $?
    python3 -c "
import json;d=json.load(open('$D/s${sl}_r$r.json'));print('slots=$sl r$r', round(d['value'],1),'it/s', round(d['matvec_gbps'],1),'GB/s', d['check']['relres'])"
  done
done
