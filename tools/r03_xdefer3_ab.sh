#!/bin/bash
# Poisson m=8192: x every iteration (0), every other (1, the default), every
# third (3, a third p slab), interleaved (three variants: no aliasing with a
# process-to-process alternation); the Poisson tests and the m=8192 bit check first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q --timeout 600 --timeout-method thread -m gpu -k poisson \
    -p no:cacheprovider > gpurun_out/r03_xdefer3_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_xdefer3_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for d in 0 1 3; do
    CGX_POISSON_XDEFER=$d timeout -k 10 240 python bench.py --workload poisson --no-cpu --steps 300 \
        > gpurun_out/r03_xd3.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_xd3.json'))
print(json.dumps({'xdefer': '$d', 'round': $r, 'it_s': round(d['value'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_xdefer3_ab.jsonl
  done
done
CGX_POISSON_XDEFER=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xd3/prof_kt -o kt --output-format csv -- \
    python bench.py --workload poisson --no-cpu > gpurun_out/xd3_kt.json 2> gpurun_out/xd3_kt.err || exit $?
