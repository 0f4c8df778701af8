#!/bin/bash
# symmetric storage: parity tests, then the bench at N=65536 and 16384 (two rounds)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu \
    -k "symmetric" -p no:cacheprovider > gpurun_out/r03e_sym_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03e_sym_tests.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for n in 65536 16384; do
    timeout -k 10 240 python bench.py --workload symmetric --size $n --no-cpu --steps 50 \
        > gpurun_out/r03e_sym_n${n}_r${r}.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03e_sym_n${n}_r${r}.json'))
print($n, $r, round(d['value'],1), 'it/s', round(d['matvec_ms'],4), 'ms', round(d['roofline']['achieved'],1), 'GB/s')"
  done
done
