#!/bin/bash
# Poisson configs[4]: x updated every other iteration (CGX_POISSON_XDEFER=1,
# the default) against every iteration -- the Poisson -m gpu tests, then bench
# lines interleaved (variant "own": each xr kernel on its own occupancy's
# grid, CGX_XR_OWN_GRID=1), then a kernel trace of each.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/r03_xdefer_bits.py 8192 > gpurun_out/r03_xdefer_bits.log 2>&1 || exit $?
cat gpurun_out/r03_xdefer_bits.log
timeout -k 10 600 python -u -m pytest tests -v --timeout 500 --timeout-method thread -m gpu -k "poisson" \
    -p no:cacheprovider > gpurun_out/r03_xdefer_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03_xdefer_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1 own; do
    if [ $v = own ]; then d=1; og=1; else d=$v; og=0; fi
    CGX_POISSON_XDEFER=$d CGX_XR_OWN_GRID=$og timeout -k 10 240 python bench.py --workload poisson --no-cpu \
        --steps 200 > gpurun_out/r03_xdefer${v}_r${r}.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_xdefer${v}_r${r}.json'))
print(json.dumps({'xdefer': '$v', 'round': $r, 'it_s': round(d['value'],1), 'iteration_gbps': round(d['iteration_gbps'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_xdefer_ab.jsonl
  done
done
for d in 0 1; do
  D=gpurun_out/xdefer$d
  mkdir -p $D
  CGX_POISSON_XDEFER=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_kt -o kt --output-format csv -- \
      python bench.py --workload poisson --no-cpu > $D/kt.json 2> $D/kt.err || exit $?
done
