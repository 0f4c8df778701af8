#!/bin/bash
# Measurement script for one round (run on the GPU box from the repo root):
#   gpurun -- 'bash tools/profile_round.sh'
# 1. the default bench line (dense N=65536, 1 GPU, with cpu_baseline)
# 2. rocprofv3 --kernel-trace --stats of the same bench command (no CPU leg)
# 3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the traffic figure
# Every GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o kt --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_kt.json 2> $OUT/bench_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o fetch --output-format csv -- \
    python bench.py --steps 4 --warmup 1 --no-cpu > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o write --output-format csv -- \
    python bench.py --steps 4 --warmup 1 --no-cpu > $OUT/bench_write.json 2> $OUT/bench_write.err
cat $OUT/bench_default.json
