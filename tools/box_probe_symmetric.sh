#!/bin/bash
# What differs on a box where k_symv_f64 reads 6.26 TB/s instead of 6.9:
# the GPU's partition modes and clocks, the symmetric and dense bench, and the
# pure region-read pattern (tools/microbench/hbm_region_read, built in-tree).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r03_box_probe.txt
: > $O
(timeout 60 amd-smi static --partition 2>&1; timeout 60 amd-smi metric --clock 2>&1 | head -60;
 timeout 60 rocm-smi --showmemorypartition --showcomputepartition 2>&1) >> $O
timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 50 > gpurun_out/r03_probe_sym.json || exit $?
timeout -k 10 240 python bench.py --no-cpu --steps 20 > gpurun_out/r03_probe_dense.json || exit $?
timeout -k 10 300 tools/microbench/_bin/hbm_region_read 16 > gpurun_out/r03_probe_region.txt 2>&1 || exit $?
python3 -c "
import json
s=json.load(open('gpurun_out/r03_probe_sym.json')); d=json.load(open('gpurun_out/r03_probe_dense.json'))
print(json.dumps({'sym_it_s': round(s['value'],1), 'sym_gbps': round(s['roofline']['achieved'],1), 'dense_it_s': round(d['value'],1), 'dense_gbps': round(d['roofline']['achieved'],1)}))" | tee -a $O
cat gpurun_out/r03_probe_region.txt >> $O
