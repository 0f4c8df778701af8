#!/bin/bash
# k_symv_f64 with DPP lane exchanges instead of ds_bpermute: the symmetric
# tests, then bench lines interleaved with the HEAD build (tools/ab_lib.py).
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_symdpp
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_symmetric.py -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/tests.log 2>&1
rc=$?
tail -2 $D/tests.log
[ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python tools/ab_lib.py ab/libcgx_head.so bench.py --workload symmetric --no-cpu --steps 30 \
      > $D/head_r$r.json 2> /dev/null || exit $?
  timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/dpp_r$r.json 2> /dev/null || exit $?
  for v in head dpp; do python3 -c "
import json;d=json.load(open('$D/${v}_r$r.json'));print('$v r$r', round(d['value'],1),'it/s', round(d['matvec_gbps'],1),'GB/s', d['check']['relres'])"; done
done
