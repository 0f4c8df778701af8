#!/bin/bash
# CGX_SYMMETRIC at N=65536, the same (default) kernel in consecutive bench
# processes: does the rate alternate process to process (slow, fast, ...)
# with the default 3 s settle, and with a 15 s one?
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in 3 3 3 3 3 3 15 15 15 15; do
  timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 50 --settle $st > gpurun_out/r03_sympar.json || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/r03_sympar.json'))
print(json.dumps({'settle_s': $st, 'it_s': round(d['value'],1), 'gbps': round(d['roofline']['achieved'],1)}))" | tee -a gpurun_out/r03_sym_parity.jsonl
done
