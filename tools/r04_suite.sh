# the whole -m gpu suite on the current tree (round 4)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu \
    --durations=25 -p no:cacheprovider > gpurun_out/r04_suite2.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_suite2.log | tail -15
exit $rc
