#!/bin/bash
# round 4, step 18: the overlap's wrapped "rest" matVec as one pipeline
# (pick_mv_wrap) against two (CGX_MV_WRAP_SPLIT=1): the bitwise tests, then
# one rank's iteration at G = 4 / 8 without the collectives, interleaved, and
# a kernel trace of each at G = 8
set -u
export TMPDIR=/tmp
D=gpurun_out/r04_wrap
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_multirank.py -m gpu -q --timeout 250 \
    --timeout-method thread -k "wrapped_column or local_exchange or world8 or shards_f64" > $D/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $D/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
: > $D/rank_iteration.jsonl
for r in 0 1 2; do
    for g in 4 8; do
        for split in 0 1; do
            CGX_MV_WRAP_SPLIT=$split timeout -k 10 120 tools/microbench/_bin/rank_iteration $g 60 \
                | sed "s/^{/{\"wrap_split\": $split, \"round\": $r, /" >> $D/rank_iteration.jsonl || exit 1
        done
    done
done
cat $D/rank_iteration.jsonl
for split in 0 1; do
    CGX_MV_WRAP_SPLIT=$split timeout -k 10 120 rocprofv3 --kernel-trace -d $D/kt_split$split -o kt --output-format csv -- \
        tools/microbench/_bin/rank_iteration 8 60 > /dev/null || exit 1
done
for split in 0 1; do find $D/kt_split$split -name "*kernel_trace.csv" | while read f; do echo "== split $split"; python3 -c "
import csv,re,collections
rows=sorted(csv.DictReader(open('$f')), key=lambda r:int(r['Start_Timestamp']))[-120:]
d=collections.defaultdict(list)
for r in rows:
    n=re.search(r'(k_\w+)(<[^>]*>)?', r['Kernel_Name'])
    if n: d[n.group(0)].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000)
for k,v in d.items():
    v=sorted(v); print(k, len(v), 'min', round(v[0],1), 'median', round(v[len(v)//2],1), 'max', round(v[-1],1))"; done; done
