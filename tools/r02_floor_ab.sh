set -euo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 250 --timeout-method thread -k "two_launch or p2p_local or device_gated or solve_in_pieces or zero_x0 or timing_events or f64_parity or max_iter" > gpurun_out/r02_fusep_tests.log 2>&1
for rep in 1 2; do
  for f in 0 1; do
    CGX_FUSE_P=$f timeout -k 10 200 python tools/iter_floor.py 64 512 2048 4096 8192 >> gpurun_out/r02_iter_floor_ab.jsonl 2>&1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o small --output-format csv -- python tools/iter_floor.py 512 2048 8192 > gpurun_out/r02_iter_floor_rocprof.jsonl 2>&1
