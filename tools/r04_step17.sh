#!/bin/bash
# round 4, step 17: the pipelined xr kernel with an item's last two p rows
# loaded with its first step (CGX_EARLY_TAIL): the bitwise tests, an
# interleaved A/B, DRAM requests per kernel with and without it
set -u
export TMPDIR=/tmp
D=gpurun_out/r04_et
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_solver.py -m gpu -q --timeout 300 --timeout-method thread \
    -k "pipelined or x_every_other or configs4" > $D/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $D/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_variants.py --rounds 3 --args "--workload poisson --steps 300" \
    --variant et1= --variant et0=CGX_EARLY_TAIL=0 --variant et1xr4=CGX_XR_PIPE=4 --variant et0xr4=CGX_EARLY_TAIL=0,CGX_XR_PIPE=4 \
    > $D/ab.jsonl || exit 1
python3 -c "
import json
for l in open('$D/ab.jsonl'):
    d=json.loads(l); print(d.get('variant'), d.get('round'), d.get('value'))"
for et in 1 0; do
    export CGX_EARLY_TAIL=$et
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum -d $D/poisson_et${et}_A -o p \
        --output-format csv -- python3 bench.py --workload poisson --no-cpu --phases off --steps 6 --warmup 1 \
        > $D/poisson_et${et}_A.json 2> $D/poisson_et${et}_A.err || exit $?
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/kt_et$et -o kt --output-format csv -- \
        python3 bench.py --workload poisson --no-cpu --steps 150 --warmup 3 > $D/kt_et$et.json 2> $D/kt_et$et.err || exit $?
done
unset CGX_EARLY_TAIL
python3 tools/pmc_sizes.py --dir $D > $D/pmc_sizes.json || exit $?
python3 -c "
import json
d=json.load(open('$D/pmc_sizes.json'))
for w,v in d['workloads'].items():
    for k,e in v['kernels'].items():
        if 'poisson' in k: print(w, k, round(e.get('dram_over_algorithmic',0),4))"
for et in 1 0; do find $D/kt_et$et -name "*kernel_stats.csv" | while read f; do echo "== et$et"; python3 -c "
import csv,re
for r in csv.DictReader(open('$f')):
    k=re.search(r'k_poisson\w*(<[^>]*>)?', r['Name'])
    if k: print(k.group(0), r['Calls'], round(float(r['AverageNs'])/1000,1))"; done; done
