#!/bin/bash
# fold parity tests, then the iteration floor of the launch forms
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu \
    -k "two_launch_iteration_bitwise" -p no:cacheprovider > gpurun_out/r03d_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03d_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/r03_floor.py 2 "${1:-2048,4096,8192}" > gpurun_out/r03d_floor.jsonl || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/r03d_floor.jsonl"):
    d = json.loads(l)
    print(d["round"], d["n"], d["form"], round(d["us_per_iter"], 2), d["phases_median_us"])
PY
