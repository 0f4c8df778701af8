# round 4, step 5: host cost per HIP call (kernel-argument size, streams,
# events); the Poisson pipelined xr kernel per x mode (rows per step 4 for the
# no-x kernel, 2 or 4 for the catch-up), interleaved, then a kernel trace of
# each variant
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/microbench/_bin/host_enqueue > gpurun_out/r04_host_enqueue.json || exit 1
cat gpurun_out/r04_host_enqueue.json
timeout -k 10 400 python -u tools/ab_variants.py --rounds 2 --args "--workload poisson --steps 300" \
    --variant default= --variant xr4=CGX_XR_PIPE=4 --variant xr4c2=CGX_XR_PIPE=4,CGX_XR_PIPE_CATCHUP=2 \
    --variant xr4c0=CGX_XR_PIPE=4,CGX_XR_PIPE_CATCHUP=9 > gpurun_out/r04_poisson_ab2.jsonl || exit 1
cat gpurun_out/r04_poisson_ab2.jsonl
for v in default xr4 xr4c2; do
  e="CGX_XR_PIPE=0"; [ $v = xr4 ] && e="CGX_XR_PIPE=4"; [ $v = xr4c2 ] && e="CGX_XR_PIPE=4 CGX_XR_PIPE_CATCHUP=2"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_pois_kt_$v -o kt --output-format csv -- \
      python bench.py --workload poisson --no-cpu --steps 150 > gpurun_out/r04_pois_kt_$v.json 2>&1 || exit 1
done
