#!/bin/bash
# The distinct-device tests (tests/test_gpu_multidevice.py) on a one-GPU box:
# CGX_TEST_MULTIDEVICE_REHEARSAL=1 makes every "device" device 0 (row blocks
# [0]*G, rank processes with their own NCCL_HOSTID), so the tests' own code
# paths run before the first node with several GPUs does.  Not a multi-GPU
# result: xGMI and peer access are not exercised.
#   gpurun -- 'bash tools/multidevice_rehearsal.sh'
set -euo pipefail
export TMPDIR=/tmp CGX_TEST_MULTIDEVICE_REHEARSAL=1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_multidevice.py -m gpu -x -v --timeout 900 \
    --timeout-method thread > gpurun_out/multidevice_rehearsal.log 2>&1 || { tail -60 gpurun_out/multidevice_rehearsal.log; exit 1; }
tail -30 gpurun_out/multidevice_rehearsal.log
