#!/bin/bash
# Round-2 re-measure of the small-system iteration after the one-step p pass
# (k_update_xrp_f64's last block issues all of its p/r loads at once) and the
# R = 1 matVec plan for 4096-8192 columns: bitwise tests, the per-iteration
# floor, and a rocprofv3 kernel trace at n = 2048 / 4096 / 8192.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 250 --timeout-method thread \
    -k "two_launch or device_gated or solve_in_pieces" > $OUT/r02_ppass_tests.log 2>&1
rm -f $OUT/r02_iter_floor_ppass.jsonl
for rep in 1 2; do
  timeout -k 10 200 python tools/iter_floor.py 512 1024 2048 4096 8192 >> $OUT/r02_iter_floor_ppass.jsonl 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_ppass -o small --output-format csv -- \
    python tools/iter_floor.py 2048 4096 8192 > $OUT/r02_iter_floor_ppass_rocprof.jsonl 2>&1
