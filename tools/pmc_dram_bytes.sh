#!/bin/bash
# Calibrated HBM bytes per kernel (MI355X_MICROARCH.md: FETCH_SIZE is only
# calibrated for 16-B-per-lane streaming reads).  For the dense, symmetric
# and Poisson bench workloads, three --pmc passes each:
#   A: TCC_EA0_RDREQ_DRAM_32B_sum, TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
#      (DRAM-bound requests in 32-B units: one 64-B request counts 2)
#   B: TCC_EA0_RDREQ_{32B,64B,128B}_sum, TCC_EA0_RDREQ_sum (request sizes)
#   C: FETCH_SIZE (the doubled figure DESIGN quoted so far)
# Summary: tools/pmc_sizes.py -> gpurun_out/r03_pmc_sizes.json.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsz
run() {  # workload tag pass counters...
  local w=$1 tag=$2 pass=$3; shift 3
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmcsz/${tag}_$pass -o p --output-format csv -- \
      python3 bench.py --workload $w --no-cpu --phases off --steps 4 --warmup 1 > gpurun_out/pmcsz/${tag}_$pass.json \
      2> gpurun_out/pmcsz/${tag}_$pass.err || exit $?
}
for w in dense symmetric poisson; do
  run $w $w A TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
  run $w $w B TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
  run $w $w C FETCH_SIZE
done
python3 tools/pmc_sizes.py --dir gpurun_out/pmcsz > gpurun_out/r03_pmc_sizes.json
# kernel split of the symmetric matVec (tiles kernel vs reduce)
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcsz/sym_kt -o kt --output-format csv -- \
    python3 bench.py --workload symmetric --no-cpu --steps 20 > gpurun_out/pmcsz/sym_kt.json 2> gpurun_out/pmcsz/sym_kt.err || exit $?
