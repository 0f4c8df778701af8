#!/bin/bash
# Poisson configs[4]: XCD bands (CGX_POISSON_BANDS=1) against the strip-
# fastest grid-stride hand-out -- bench lines interleaved, then a kernel trace
# and the FETCH_SIZE / WRITE_SIZE passes of each (tools/pmc_poisson.py).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for b in 0 1; do
    CGX_POISSON_BANDS=$b timeout -k 10 240 python bench.py --workload poisson --no-cpu --steps 200 \
        > gpurun_out/r03_pois_b${b}_r${r}.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_pois_b${b}_r${r}.json'))
print('bands=$b round=$r', round(d['value'],1), 'it/s', round(d['iteration_gbps'],1), 'GB/s/iter')"
  done
done
for b in 0 1; do
  D=gpurun_out/pois_b$b
  mkdir -p $D
  export CGX_POISSON_BANDS=$b
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_pois_kt -o kt --output-format csv -- \
      python bench.py --workload poisson --no-cpu > $D/kt.json 2> $D/kt.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/prof_pois_fetch -o fetch --output-format csv -- \
      python bench.py --workload poisson --no-cpu --steps 4 --warmup 1 > /dev/null 2> $D/fetch.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/prof_pois_write -o write --output-format csv -- \
      python bench.py --workload poisson --no-cpu --steps 4 --warmup 1 > /dev/null 2> $D/write.err || exit $?
  python3 tools/pmc_poisson.py --tag r03_bands$b --m 8192 --dir $D > /dev/null || exit $?
  python3 -c "
import json;d=json.load(open('profiles/r03_bands${b}_pmc_poisson_m8192.json'))
for k,v in d['kernels'].items(): print('bands=$b', k, round(v['hbm_B_per_point'],2), 'B/pt of', v['algorithmic_B_per_point'], round(v['kernel_trace_avg_us'],1), 'us')"
done
