#!/bin/bash
# configs[1] (N=16384, 1 GPU): kernel stats and the two PMC passes for roofline.traffic
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof16_kt -o kt --output-format csv -- \
    python bench.py --n 16384 --steps 50 --warmup 5 --no-cpu > $OUT/bench16_kt.json 2> $OUT/bench16_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof16_fetch -o fetch --output-format csv -- \
    python bench.py --n 16384 --steps 8 --warmup 1 --no-cpu > $OUT/bench16_fetch.json 2> $OUT/bench16_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof16_write -o write --output-format csv -- \
    python bench.py --n 16384 --steps 8 --warmup 1 --no-cpu > $OUT/bench16_write.json 2> $OUT/bench16_write.err
timeout -k 10 300 python bench.py --n 16384 --steps 200 --warmup 10 > $OUT/bench16.json 2> $OUT/bench16.err
