#!/bin/bash
# One pipeline across the column wrap of the overlap path's "rest" matVec:
# the rank-mode and multi-shard parity tests, then one rank's iteration
# without collectives (tools/microbench/rank_iteration, rank P/2 so the rest
# wraps) against the HEAD build (ab/rank_iteration_head), interleaved, and a
# kernel trace of each at G = 8.
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_wrap
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_solver.py -q --timeout 500 \
    --timeout-method thread -k "shard or rank_mode or overlap or multi or local" -p no:cacheprovider > $D/tests.log 2>&1
rc=$?
tail -3 $D/tests.log
[ $rc -le 1 ] || exit $rc
: > $D/ab.jsonl
for r in 1 2; do
  for g in 8 4 2; do
    echo "{\"build\": \"head\", \"round\": $r, \"line\": $(timeout -k 10 60 ab/rank_iteration_head $g 60)}" >> $D/ab.jsonl || exit 1
    echo "{\"build\": \"new\", \"round\": $r, \"line\": $(timeout -k 10 60 tools/microbench/rank_iteration $g 60)}" >> $D/ab.jsonl || exit 1
  done
done
cat $D/ab.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['build'], d['round'], d['line']['ranks'], d['line']['us_per_iteration_without_collectives'])"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt_head -o kt --output-format csv -- ab/rank_iteration_head 8 60 > /dev/null || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt_new -o kt --output-format csv -- tools/microbench/rank_iteration 8 60 > /dev/null || exit $?
python3 - <<'PY'
import csv
for b in ("head", "new"):
    for r in csv.DictReader(open(f"gpurun_out/r03_wrap/kt_{b}/kt_kernel_stats.csv")):
        print(b, r["Name"][:60], r["Calls"], r["AverageNs"])
PY
