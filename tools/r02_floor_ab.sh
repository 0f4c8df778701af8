#!/bin/bash
# Round-2 A/B of the small-system iteration (run on the GPU box from the repo root):
# the two-launch iteration (CGX_FUSE_P=1, default for n <= 8192) against three
# launches (CGX_FUSE_P=0), interleaved, with tools/iter_floor.py; then a
# rocprofv3 kernel trace of the default at n = 512 / 2048 / 8192.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_kernels.py -x -q --timeout 250 \
    --timeout-method thread -k "two_launch or p2p_local or device_gated or solve_in_pieces or zero_x0 or timing_events or f64_parity or max_iter or matvec" \
    > $OUT/r02_fusep_tests.log 2>&1
rm -f $OUT/r02_iter_floor_ab.jsonl
for rep in 1 2; do
  for f in 0 1; do
    CGX_FUSE_P=$f timeout -k 10 200 python tools/iter_floor.py 64 512 1024 2048 4096 8192 >> $OUT/r02_iter_floor_ab.jsonl 2>&1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_small -o small --output-format csv -- \
    python tools/iter_floor.py 512 2048 8192 > $OUT/r02_iter_floor_rocprof.jsonl 2>&1
