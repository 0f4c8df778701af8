# round 4, step 1: the solver tests (multi-shard pull exchange, plan change
# inside a solve), the new bench / fail-fast / MPI CLI tests, then the
# multi-shard floor with both exchange forms interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_mpi_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_step1_tests.log 2>&1 || { tail -30 gpurun_out/r04_step1_tests.log; exit 1; }
tail -3 gpurun_out/r04_step1_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread -k "without_launcher or fails_fast or torchrun_world2 or headline_n65536_world8 or world8" > gpurun_out/r04_step1_tests2.log 2>&1 || { tail -30 gpurun_out/r04_step1_tests2.log; exit 1; }
tail -3 gpurun_out/r04_step1_tests2.log
timeout -k 10 400 python -u tools/r04_multishard_floor.py 2 4096,65536 1,2,4,8 > gpurun_out/r04_floor_ab.jsonl || exit 1
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/r04_hiptrace_after -o run --output-format csv -- \
    python3 tools/r04_multishard_floor.py 1 4096 8 kernel > gpurun_out/r04_hiptrace_after.log 2>&1
