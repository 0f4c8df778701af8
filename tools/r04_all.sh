# round 4, everything in one box session, most important first; every GPU
# step has its own time limit and the chain stops at the first failure:
#  1. the whole -m gpu suite (the new multi-shard, plan, Poisson-pipeline,
#     bench and fail-fast tests included)
#  2. the multi-shard floor (kernel / nofuse / copy exchange, S = 1/2/4/8)
#     and a HIP API trace of S = 8 with the default exchange
#  3. the HBM stream-mix ceilings, one rank's iteration at G = 2/4/8 with its
#     kernel traces (the scale model's inputs)
#  4. the Poisson pipelined-kernel A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu \
    --durations=25 -p no:cacheprovider > gpurun_out/r04_suite.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04_suite.log | tail -15
[ $rc -le 1 ] || exit $rc   # test failures (1) still let the measurements run; a crash or time-out stops here
timeout -k 10 240 python -u tools/r04_multishard_floor.py 1 4096 1,2,4,8 > gpurun_out/r04_floor_ab.jsonl || exit 1
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/r04_hiptrace_after -o run --output-format csv -- \
    python3 tools/r04_multishard_floor.py 1 4096 8 kernel > gpurun_out/r04_hiptrace_after.log 2>&1 || exit 1
bash tools/r04_step2.sh || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --rounds 1 --args "--workload poisson --steps 300" \
    --variant default= --variant xr2=CGX_XR_PIPE=2 --variant xr4=CGX_XR_PIPE=4 \
    --variant xr2p2=CGX_XR_PIPE=2,CGX_P_PIPE=2 --variant xr2p4=CGX_XR_PIPE=2,CGX_P_PIPE=4 \
    > gpurun_out/r04_poisson_ab.jsonl || exit 1
cat gpurun_out/r04_poisson_ab.jsonl
