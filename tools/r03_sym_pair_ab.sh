#!/bin/bash
# CGX_SYMMETRIC: one column-partial barrier per pair of units (CGX_SYM_PAIR=1)
# against one per unit -- the symmetric -m gpu tests under the pair kernel,
# then bench lines interleaved at N=65536 and 16384 (relres equal = same bits).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
CGX_SYM_PAIR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_symmetric.py -q --timeout 300 \
    --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/r03_sym_pair_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_sym_pair_tests.log
[ $rc -eq 0 ] || exit $rc
for n in 65536 32768 16384; do
  for r in 1 2; do
    for v in 0 1; do
      CGX_SYM_PAIR=$v timeout -k 10 240 python bench.py --workload symmetric --n $n --no-cpu --steps 50 \
          > gpurun_out/r03_sympair${v}_n${n}_r$r.json || exit $?
      python3 -c "
import json;d=json.load(open('gpurun_out/r03_sympair${v}_n${n}_r$r.json'))
print(json.dumps({'pair': $v, 'n': $n, 'round': $r, 'it_s': round(d['value'],1), 'gbps': round(d['roofline']['achieved'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_sym_pair_ab.jsonl
    done
  done
done
