#!/bin/bash
# k_matvec_small_f64 (p staged in LDS, n = 2048..8192 on one GPU): the
# small-system parity tests, then the iteration floor of every launch form
# with and without it, and the block-size / chunk variants of the fold.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu \
    -k "two_launch or published or small or n2048 or n4096 or n8192 or plan" -p no:cacheprovider \
    > gpurun_out/r03s_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03s_tests.log
[ $rc -le 1 ] || exit $rc
R03_SMALL_VARIANTS=1 timeout -k 10 400 python tools/r03_floor.py 2 "${1:-2048,4096,8192}" > gpurun_out/r03s_floor.jsonl || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/r03s_floor.jsonl"):
    d = json.loads(l)
    ph = d["phases_median_us"]
    print(d["round"], d["n"], d["form"], round(d["us_per_iter"], 2), "iter", ph.get("iteration"), "mv", ph.get("matvec"))
PY
exit $rc
