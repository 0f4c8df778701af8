#!/bin/bash
# configs[3]'s system as upper-triangle tiles streamed from host memory with
# an HBM budget for the first tiles (bench.py --workload stream_symmetric
# --resident-gb): 0 / 32 / 64 GB of the 68.7 GB of tiles.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
for gb in 0 32 64; do
  timeout -k 10 300 python bench.py --workload stream_symmetric --steps 2 --warmup 1 --resident-gb $gb \
      > $OUT/r02_bench_stream_sym_resident_${gb}.json 2> $OUT/r02_bench_stream_sym_resident_${gb}.err
done
