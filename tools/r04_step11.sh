#!/bin/bash
# round 4, step 11: the Poisson MALL tail (CGX_MALL_TAIL_MB: the last items'
# output stores default-policy, so the next kernel, walking the other way,
# finds them in the memory-side cache): the bitwise tests, an interleaved A/B
# over the tail size, a kernel trace at the best candidate
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -m gpu -q --timeout 200 --timeout-method thread \
    -k "mall_tail" > gpurun_out/r04_step11_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_step11_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/ab_variants.py --rounds 3 --args "--workload poisson --steps 300" \
    --variant t0=CGX_MALL_TAIL_MB=0 --variant t32=CGX_MALL_TAIL_MB=32 --variant t64=CGX_MALL_TAIL_MB=64 \
    --variant t128=CGX_MALL_TAIL_MB=128 --variant t192=CGX_MALL_TAIL_MB=192 --variant t256=CGX_MALL_TAIL_MB=256 \
    > gpurun_out/r04_poisson_mall_ab.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r04_poisson_mall_ab.jsonl'):
    d=json.loads(l); print(d.get('variant'), d.get('round'), d.get('value'))"
for t in 0 128; do
    export CGX_MALL_TAIL_MB=$t
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_step11_t$t -o kt --output-format csv -- \
        python3 bench.py --workload poisson --steps 150 --warmup 3 --no-cpu > gpurun_out/r04_step11_t$t.log 2>&1 || exit 1
done
unset CGX_MALL_TAIL_MB
find gpurun_out/r04_step11_t* -name "*kernel_stats.csv" | while read f; do echo "== $f"; python3 -c "
import csv,re
for r in csv.DictReader(open('$f')):
    k=re.search(r'k_poisson\w*(<[^>]*>)?', r['Name'])
    if k: print(k.group(0), r['Calls'], round(float(r['AverageNs'])/1000,1))"; done
