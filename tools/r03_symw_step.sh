#!/bin/bash
# k_symv_f64 with one stream per wave (no LDS, no barrier): the symmetric
# tests, then bench lines interleaved with the HEAD build (ab/libcgx_head.so,
# tools/ab_lib.py), a kernel trace and the DRAM-byte pass of the new kernel.
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_symw
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_symmetric.py -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/tests.log 2>&1
rc=$?
tail -3 $D/tests.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python tools/ab_lib.py ab/libcgx_head.so bench.py --workload symmetric --no-cpu --steps 30 \
      > $D/head_r$r.json 2> $D/head_r$r.err || exit $?
  timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/new_r$r.json 2> $D/new_r$r.err || exit $?
  for v in head new; do python3 -c "
import json;d=json.load(open('$D/${v}_r$r.json'));print('$v r$r', round(d['value'],1),'it/s', round(d['matvec_gbps'],1),'GB/s', d['check']['relres'])"; done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- \
    python3 bench.py --workload symmetric --no-cpu --steps 20 > $D/kt.json 2> $D/kt.err || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum -d $D/pmc -o p \
    --output-format csv -- python3 bench.py --workload symmetric --no-cpu --steps 4 --warmup 1 > /dev/null 2> $D/pmc.err || exit $?
python3 - <<'PY'
import csv, glob
D = "gpurun_out/r03_symw"
for r in csv.DictReader(open(f"{D}/kt/kt_kernel_stats.csv")):
    if "symv" in r["Name"]:
        print(r["Name"][:40], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
v = {}
for f in glob.glob(f"{D}/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_symv_f64" in r["Kernel_Name"]:
            v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for c, x in v.items():
    print(c, 32 * sum(x) / len(x))
PY
