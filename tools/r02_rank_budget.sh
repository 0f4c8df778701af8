#!/bin/bash
# The non-communication budget of one rank's iteration at G = 2/4/8 (N=65536):
# tools/microbench/rank_iteration timed, then under rocprofv3 --kernel-trace.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
rm -f $OUT/r02_rank_iteration.jsonl
for g in 8 4 2; do
  timeout -k 10 120 tools/microbench/rank_iteration $g 60 >> $OUT/r02_rank_iteration.jsonl
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_rank8 -o rank8 --output-format csv -- \
    tools/microbench/rank_iteration 8 60 > $OUT/r02_rank_iteration_rocprof.jsonl
