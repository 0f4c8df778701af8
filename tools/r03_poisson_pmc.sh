#!/bin/bash
# Poisson configs[4] with x every other iteration: the -m gpu Poisson tests
# (the vectorised x flush), the DRAM-request passes of tools/r03_pmc_sizes.sh
# for the Poisson workload only, and configs[1] (N=16384) with the p update
# folded into the matVec (CGX_FUSE_P=1 CGX_FOLD_P=1) against the default.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsz
timeout -k 10 600 python -u -m pytest tests -q --timeout 500 --timeout-method thread -m gpu -k "poisson" \
    -p no:cacheprovider > gpurun_out/r03_poisson_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03_poisson_tests.log
[ $rc -eq 0 ] || exit $rc
run() {  # workload tag pass counters...
  local w=$1 tag=$2 pass=$3; shift 3
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmcsz/${tag}_$pass -o p --output-format csv -- \
      python3 bench.py --workload $w --no-cpu --phases off --steps 4 --warmup 1 > gpurun_out/pmcsz/${tag}_$pass.json \
      2> gpurun_out/pmcsz/${tag}_$pass.err || exit $?
}
run poisson poisson A TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
run poisson poisson B TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
run poisson poisson C FETCH_SIZE
python3 tools/pmc_sizes.py --dir gpurun_out/pmcsz > gpurun_out/r03_pmc_sizes_poisson.json
for r in 1 2; do
  for f in 0 1; do
    if [ $f = 1 ]; then export CGX_FUSE_P=1 CGX_FOLD_P=1; else unset CGX_FUSE_P CGX_FOLD_P; fi
    timeout -k 10 240 python bench.py --n 16384 --no-cpu --steps 300 > gpurun_out/r03_n16384_fold${f}_r$r.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03_n16384_fold${f}_r$r.json'))
print(json.dumps({'fold': $f, 'round': $r, 'it_s': round(d['value'],1), 'matvec_gbps': round(d['matvec_gbps'],1), 'relres': d['check']['relres']}))" | tee -a gpurun_out/r03_n16384_fold_ab.jsonl
  done
done
