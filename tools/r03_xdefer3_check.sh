#!/bin/bash
# x every third iteration as the default: the Poisson tests, then the default
# Poisson bench line (the bit check at m=8192 against every-iteration x).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q --timeout 600 --timeout-method thread -m gpu -k poisson \
    -p no:cacheprovider > gpurun_out/r03_xdefer3_default_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_xdefer3_default_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/r03_xdefer_bits.py 8192 > gpurun_out/r03_xdefer3_bits.log 2>&1 || exit $?
cat gpurun_out/r03_xdefer3_bits.log
timeout -k 10 240 python bench.py --workload poisson > gpurun_out/r03_bench_poisson_default.json || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/r03_bench_poisson_default.json'))
print(round(d['value'],1), round(d['iteration_gbps'],1), d['roofline']['achieved'], d['check'])"
