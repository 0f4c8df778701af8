#!/bin/bash
# One gpurun call: targeted -m gpu tests, then (unless the tests crashed or
# timed out) the default bench with the phase breakdown on.
#   tools/r03_gpu_step.sh "<pytest -k expression>" <tag>
set -u
K="$1"; TAG="$2"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v --timeout 900 --timeout-method thread -m gpu -k "$K" \
    --durations=25 -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --phases on > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
brc=$?
echo "bench rc=$brc"; cat gpurun_out/${TAG}_bench.json | head -c 600
exit $rc
