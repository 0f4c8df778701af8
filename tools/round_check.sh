#!/bin/bash
# End-of-round check on one GPU box (repo root): the whole -m gpu suite, then
# tools/profile_round.sh (default bench line, rocprofv3 kernel trace of the
# same command, FETCH_SIZE / WRITE_SIZE passes).  Every GPU step has its own
# time limit; the chain stops at a crash or a time-out.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q --timeout 800 --timeout-method thread -m gpu \
    --durations=30 -p no:cacheprovider > gpurun_out/suite.log 2>&1
rc=$?
tail -4 gpurun_out/suite.log
[ $rc -le 1 ] || exit $rc
bash tools/profile_round.sh || exit $?
exit $rc
