#!/bin/bash
# round 4, step 9: pipelined Poisson kernels with the side points loaded by the
# outer waves only (CGX_PIPE_SIDE_EDGE): the pipelined-kernel tests, then an
# interleaved A/B of the kernel choices, then a kernel trace of the candidates
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -m gpu -q --timeout 200 --timeout-method thread \
    -k "pipelined or x_every_other" > gpurun_out/r04_step9_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_step9_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_variants.py --rounds 3 --args "--workload poisson --steps 300" \
    --variant default= --variant allside=CGX_PIPE_SIDE_EDGE=0 --variant xr4=CGX_XR_PIPE=4 \
    --variant p4=CGX_P_PIPE=4 --variant xr4p4=CGX_XR_PIPE=4,CGX_P_PIPE=4 --variant xr2p2=CGX_XR_PIPE=2,CGX_P_PIPE=2 \
    > gpurun_out/r04_poisson_side_ab.jsonl || exit 1
cat gpurun_out/r04_poisson_side_ab.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('round'), d.get('value'))"
for v in default xr4p4; do
    if [ $v = xr4p4 ]; then export CGX_XR_PIPE=4 CGX_P_PIPE=4; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_side_$v -o run -- \
        python3 bench.py --workload poisson --steps 150 --warmup 3 --no-cpu > gpurun_out/r04_prof_side_$v.log 2>&1 || exit 1
    unset CGX_XR_PIPE CGX_P_PIPE
done
find gpurun_out/r04_prof_side_* -name "*kernel_stats.csv" | while read f; do echo "== $f"; python3 -c "
import csv,re
for r in csv.DictReader(open('$f')):
    k=re.search(r'k_poisson\w*(<[^>]*>)?', r['Name'])
    if k: print(k.group(0), r['Calls'], round(float(r['AverageNs'])/1000,1))"; done
