#!/bin/bash
# CGX_SYMMETRIC at N=65536: units per block rounded up to an odd count
# (CGX_SYM_PER_ODD=1) against the default, in consecutive processes (three of
# each, alternating), with the symmetric tests under the odd count first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
CGX_SYM_PER_ODD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_symmetric.py -q --timeout 300 \
    --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/r03_sym_odd_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_sym_odd_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 1 0 0 1 1 0; do
  CGX_SYM_PER_ODD=$v timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 50 > gpurun_out/r03_symodd.json || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/r03_symodd.json'))
print(json.dumps({'per_odd': $v, 'it_s': round(d['value'],1), 'gbps': round(d['roofline']['achieved'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_sym_odd_ab.jsonl
done
