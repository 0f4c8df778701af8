# round 4, step 6: one enqueuing thread per row block (cgx_local_mt.hip):
# the multi-shard tests, then the floor with the threaded / one-thread /
# nofuse / copy forms, S = 1/2/4/8 at N = 4096 (and S = 8 at N = 65536)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_multirank.py -m gpu -q \
    --timeout 300 --timeout-method thread \
    -k "shards or local_exchange or headline_n65536_world8 or device_generator or set_rows or phase_times or zero_x0 or indefinite or without_launcher" \
    > gpurun_out/r04_step6_tests.log 2>&1 && timeout -k 10 300 python -u -m pytest tests/test_gpu_cli.py -m gpu -q \
    --timeout 200 --timeout-method thread >> gpurun_out/r04_step6_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_step6_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/r04_multishard_floor.py 2 4096 1,2,4,8 > gpurun_out/r04_floor_mt.jsonl || exit 1
timeout -k 10 300 python -u tools/r04_multishard_floor.py 1 65536 8 kernel,onethread > gpurun_out/r04_floor_mt_65536.jsonl || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/r04_floor_mt.jsonl", "gpurun_out/r04_floor_mt_65536.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(d["n"], d["shards"], d["exchange"], "enq", d["enqueue_us"], "enq10", d["enqueue_10_us"], "wall", d["wall_us"])
PY
timeout -k 10 400 python -u tools/ab_variants.py --rounds 2 --args "--workload poisson --steps 300" \
    --variant default= --variant g1024=CGX_STENCIL_BLOCKS=1024 \
    --variant g1024q=CGX_STENCIL_BLOCKS=1024,CGX_XR3_QUARTER=1 --variant q=CGX_XR3_QUARTER=1 \
    > gpurun_out/r04_poisson_grid_ab.jsonl || exit 1
cat gpurun_out/r04_poisson_grid_ab.jsonl
