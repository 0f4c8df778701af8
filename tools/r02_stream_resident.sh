#!/bin/bash
# configs[3] (N=131072 fp64, A in pinned host memory) with an HBM budget for
# the first rows of A (bench.py --resident-gb, CGX_STREAM_RESIDENT_MB): the
# streamed-with-resident tests, then the bench at 0 / 64 / 120 GB resident.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 250 --timeout-method thread \
    -k "host_streamed" > $OUT/r02_resident_tests.log 2>&1
for gb in 0 64 120; do
  timeout -k 10 300 python bench.py --workload stream --steps 2 --warmup 1 --resident-gb $gb \
      > $OUT/r02_bench_stream_resident_${gb}.json 2> $OUT/r02_bench_stream_resident_${gb}.err
done
