# round 4, step 7: Poisson -- the pipelined catch-up kernel alone (c4) and
# both pipelined xr kernels (xr4) against the default, three interleaved
# rounds; then the round's default bench line with its rocprof kernel trace
# and PMC passes (tools/profile_round.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_variants.py --rounds 3 --args "--workload poisson --steps 400" \
    --variant default= --variant xr4=CGX_XR_PIPE=4 --variant c4=CGX_XR_PIPE_CATCHUP=4 \
    > gpurun_out/r04_poisson_ab3.jsonl || exit 1
cat gpurun_out/r04_poisson_ab3.jsonl
bash tools/profile_round.sh || exit 1
