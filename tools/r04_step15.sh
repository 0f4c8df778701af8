#!/bin/bash
# round 4, step 15: Poisson on the final tree -- the bench line, a kernel
# trace, and the calibrated DRAM-request passes (as tools/pmc_dram_bytes.sh)
# on the same box
set -u
export TMPDIR=/tmp
D=gpurun_out/r04_pois_final
mkdir -p $D
timeout -k 10 120 python3 bench.py --workload poisson --no-cpu --steps 300 > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- \
    python3 bench.py --workload poisson --no-cpu --steps 150 --warmup 3 > $D/kt.json 2> $D/kt.err || exit $?
run() {  # pass counters...
  local pass=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $D/poisson_$pass -o p --output-format csv -- \
      python3 bench.py --workload poisson --no-cpu --phases off --steps 6 --warmup 1 > $D/poisson_$pass.json \
      2> $D/poisson_$pass.err || exit $?
}
run A TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
run B TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
run C FETCH_SIZE
python3 tools/pmc_sizes.py --dir $D > $D/pmc_sizes.json || exit $?
python3 -c "
import json
print(json.load(open('$D/bench.json'))['value'])
d=json.load(open('$D/pmc_sizes.json'))
for k,v in d['workloads']['poisson']['kernels'].items():
    if 'poisson' in k: print(k, round(v.get('dram_over_algorithmic',0),4), v.get('algorithmic_B'))"
find $D/kt -name "*kernel_stats.csv" | while read f; do python3 -c "
import csv,re
for r in csv.DictReader(open('$f')):
    k=re.search(r'k_poisson\w*(<[^>]*>)?', r['Name'])
    if k: print(k.group(0), r['Calls'], round(float(r['AverageNs'])/1000,1))"; done
