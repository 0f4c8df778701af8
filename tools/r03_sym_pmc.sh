#!/bin/bash
# CGX_SYMMETRIC at N=65536 with the odd units-per-block stagger: kernel trace
# and the DRAM-request / FETCH_SIZE passes of tools/r03_pmc_sizes.sh.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsym
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcsym/kt -o kt --output-format csv -- \
    python3 bench.py --workload symmetric --no-cpu --steps 20 > gpurun_out/pmcsym/kt.json 2> gpurun_out/pmcsym/kt.err || exit $?
run() {  # workload tag pass counters...
  local w=$1 tag=$2 pass=$3; shift 3
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmcsym/${tag}_$pass -o p --output-format csv -- \
      python3 bench.py --workload $w --no-cpu --phases off --steps 4 --warmup 1 > gpurun_out/pmcsym/${tag}_$pass.json \
      2> gpurun_out/pmcsym/${tag}_$pass.err || exit $?
}
run symmetric symmetric A TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
run symmetric symmetric B TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
run symmetric symmetric C FETCH_SIZE
python3 tools/pmc_sizes.py --dir gpurun_out/pmcsym > gpurun_out/r03_pmc_sizes_symmetric.json
cat gpurun_out/pmcsym/kt.json
# other odd unit counts per block: 1027 (default), 1029, 1031, 1035 (CGX_SYM_PER_ADD2,
# an experiment knob since removed from libcgx)
for r in 1 2; do
  for a in 0 1 2 4; do
    CGX_SYM_PER_ADD2=$a timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 50 \
        > gpurun_out/r03_symper.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_symper.json'))
print(json.dumps({'per': 1027 + 2 * $a, 'round': $r, 'it_s': round(d['value'],1), 'gbps': round(d['roofline']['achieved'],1)}))" | tee -a gpurun_out/r03_sym_per_sweep.jsonl
  done
done
