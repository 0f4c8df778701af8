#!/bin/bash
# Where k_symv_f64 loses against its load pattern's 7.21-7.23 TB/s
# (profiles/r03_hbm_region_read_buffer.json): diagnostic builds with parts
# of the unit removed (results wrong by construction, timing only), built
# from a worktree copy of the source, run through tools/ab_lib.py:
#   d1: no column-partial exchange (no LDS, no barrier)
#   d2: no p loads (constants)
#   d12: both
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_symdiag
mkdir -p $D
for r in 1 2; do
  for v in cur d1 d2 d12; do
    if [ $v = cur ]; then
      timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/${v}_r$r.json 2>/dev/null || exit $?
    else
      timeout -k 10 200 python tools/ab_lib.py ab/libcgx_symv_$v.so bench.py --workload symmetric --no-cpu --steps 30 \
          > $D/${v}_r$r.json 2>/dev/null || exit $?
    fi
    python3 -c "
import json;d=json.load(open('$D/${v}_r$r.json'));print('$v r$r', round(d['value'],1),'it/s', round(d['matvec_gbps'],1),'GB/s')"
  done
done
