# round 4, step 3: Poisson m=8192 -- the software-pipelined xr kernel
# (CGX_XR_PIPE = 2 / 4 rows per step) and the x-deferred xr kernels on a grid
# of 4 blocks per CU with XM = 3 at RB / 4 (CGX_STENCIL_BLOCKS=1024
# CGX_XR3_QUARTER=1): the bitwise tests first, then interleaved bench lines,
# then a kernel trace of each variant
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "xr_pipelined or p_pipelined" > gpurun_out/r04_step3_tests.log 2>&1 || { tail -20 gpurun_out/r04_step3_tests.log; exit 1; }
tail -2 gpurun_out/r04_step3_tests.log
CGX_STENCIL_BLOCKS=1024 CGX_XR3_QUARTER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "poisson_x_every_other" > gpurun_out/r04_step3_tests2.log 2>&1 || { tail -20 gpurun_out/r04_step3_tests2.log; exit 1; }
tail -2 gpurun_out/r04_step3_tests2.log
timeout -k 10 700 python -u tools/ab_variants.py --rounds 2 --args "--workload poisson --steps 300" \
    --variant default= --variant xr2=CGX_XR_PIPE=2 --variant xr4=CGX_XR_PIPE=4 \
    --variant xr2p2=CGX_XR_PIPE=2,CGX_P_PIPE=2 --variant xr2p4=CGX_XR_PIPE=2,CGX_P_PIPE=4 \
    --variant g1024q=CGX_STENCIL_BLOCKS=1024,CGX_XR3_QUARTER=1 > gpurun_out/r04_poisson_ab.jsonl || exit 1
cat gpurun_out/r04_poisson_ab.jsonl
for v in default xr2 xr2p2; do
  e="CGX_XR_PIPE=0"; [ $v = xr2 ] && e="CGX_XR_PIPE=2"; [ $v = xr2p2 ] && e="CGX_XR_PIPE=2 CGX_P_PIPE=2"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_pois_kt_$v -o kt --output-format csv -- \
      python bench.py --workload poisson --no-cpu --steps 100 > gpurun_out/r04_pois_kt_$v.json 2>&1 || exit 1
done
