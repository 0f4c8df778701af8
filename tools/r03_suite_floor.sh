#!/bin/bash
# The whole -m gpu suite, then the small-system iteration floor (every launch
# form, the k_matvec_small_f64 block/chunk variants).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q --timeout 800 --timeout-method thread -m gpu \
    --durations=20 -p no:cacheprovider > gpurun_out/r03_suite.log 2>&1
rc=$?
tail -4 gpurun_out/r03_suite.log
[ $rc -le 1 ] || exit $rc
R03_SMALL_VARIANTS=1 timeout -k 10 400 python tools/r03_floor.py 2 "${1:-2048,4096,8192}" > gpurun_out/r03s_floor2.jsonl || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/r03s_floor2.jsonl"):
    d = json.loads(l)
    ph = d["phases_median_us"]
    print(d["round"], d["n"], d["form"], round(d["us_per_iter"], 2), "iter", ph.get("iteration"), "mv", ph.get("matvec"))
PY
exit $rc
