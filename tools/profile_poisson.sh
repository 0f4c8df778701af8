#!/bin/bash
# Poisson (configs[4]) measurement: bench line with the CPU leg, kernel trace,
# and the FETCH_SIZE / WRITE_SIZE passes (run on the GPU box from the repo root).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python bench.py --workload poisson > $OUT/bench_poisson.json 2> $OUT/bench_poisson.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_pois_kt -o kt --output-format csv -- \
    python bench.py --workload poisson --no-cpu > $OUT/bench_pois_kt.json 2> $OUT/bench_pois_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_pois_fetch -o fetch --output-format csv -- \
    python bench.py --workload poisson --no-cpu --steps 4 --warmup 1 > /dev/null 2> $OUT/bench_pois_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_pois_write -o write --output-format csv -- \
    python bench.py --workload poisson --no-cpu --steps 4 --warmup 1 > /dev/null 2> $OUT/bench_pois_write.err
cat $OUT/bench_poisson.json
