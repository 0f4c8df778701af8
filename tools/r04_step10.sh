#!/bin/bash
# round 4, step 10: on ONE box, the Poisson kernels' kernel trace (default and
# CGX_PIPE_SIDE_EDGE=0) beside the HBM ceilings of their mixes (contiguous and
# in the kernels' strip pattern), so the ratios compare like with like
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/hbm_strip_mix tools/microbench/hbm_strip_mix.hip || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/hbm_mix_peak tools/microbench/hbm_mix_peak.hip || exit 1
for v in default allside; do
    if [ $v = allside ]; then export CGX_PIPE_SIDE_EDGE=0; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_step10_$v -o kt --output-format csv -- \
        python3 bench.py --workload poisson --steps 150 --warmup 3 --no-cpu > gpurun_out/r04_step10_$v.log 2>&1 || exit 1
    unset CGX_PIPE_SIDE_EDGE
done
timeout -k 10 180 /tmp/hbm_strip_mix 8192 > gpurun_out/r04_step10_strip_mix.json || exit 1
timeout -k 10 180 /tmp/hbm_mix_peak > gpurun_out/r04_step10_hbm_mix.json || exit 1
find gpurun_out/r04_step10_* -name "*kernel_stats.csv" | while read f; do echo "== $f"; python3 -c "
import csv,re
for r in csv.DictReader(open('$f')):
    k=re.search(r'k_poisson\w*(<[^>]*>)?', r['Name'])
    if k: print(k.group(0), r['Calls'], round(float(r['AverageNs'])/1000,1))"; done
cat gpurun_out/r04_step10_strip_mix.json gpurun_out/r04_step10_hbm_mix.json
