# round 4, step 4: the multi-shard tests after the lane-parallel peer sums,
# the floor with three exchange forms (and the empty-queue enqueue), then
# step 2 (mix ceilings, rank iteration) and the Poisson pipelined-kernel A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_multirank.py -m gpu -q --timeout 300 \
    --timeout-method thread -k "shards or local_exchange or headline_n65536_world8 or world8 or device_generator or set_rows or phase_times or zero_x0 or indefinite" \
    > gpurun_out/r04_step4_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_step4_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/r04_multishard_floor.py 2 4096 1,2,4,8 > gpurun_out/r04_floor_ab2.jsonl || exit 1
timeout -k 10 300 python -u tools/r04_multishard_floor.py 1 65536 8 > gpurun_out/r04_floor_ab2_65536.jsonl || exit 1
bash tools/r04_step2.sh || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --rounds 1 --args "--workload poisson --steps 300" \
    --variant default= --variant xr2=CGX_XR_PIPE=2 --variant xr4=CGX_XR_PIPE=4 \
    --variant xr2p2=CGX_XR_PIPE=2,CGX_P_PIPE=2 --variant xr2p4=CGX_XR_PIPE=2,CGX_P_PIPE=4 \
    > gpurun_out/r04_poisson_ab.jsonl || exit 1
cat gpurun_out/r04_poisson_ab.jsonl
