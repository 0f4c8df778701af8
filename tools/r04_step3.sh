# round 4, step 3: Poisson m=8192 -- the x-deferred xr kernels on a grid of
# 4 blocks per CU (XM = 0's occupancy) instead of XM = 1's 3, with XM = 3 at
# RB / 2 or RB / 4 rows per step; the bitwise x-deferral tests under the new
# grid first, then interleaved bench lines, then a kernel trace of each
export TMPDIR=/tmp
mkdir -p gpurun_out
CGX_STENCIL_BLOCKS=1024 CGX_XR3_QUARTER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "poisson_x_every_other" > gpurun_out/r04_step3_tests.log 2>&1 || { tail -20 gpurun_out/r04_step3_tests.log; exit 1; }
tail -2 gpurun_out/r04_step3_tests.log
timeout -k 10 600 python -u tools/ab_variants.py --rounds 2 --args "--workload poisson --steps 300" \
    --variant default= --variant q=CGX_XR3_QUARTER=1 --variant g1024=CGX_STENCIL_BLOCKS=1024 \
    --variant g1024q=CGX_STENCIL_BLOCKS=1024,CGX_XR3_QUARTER=1 > gpurun_out/r04_poisson_grid_ab.jsonl || exit 1
cat gpurun_out/r04_poisson_grid_ab.jsonl
for v in default g1024q; do
  e=""; [ $v = g1024q ] && e="CGX_STENCIL_BLOCKS=1024 CGX_XR3_QUARTER=1"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_pois_kt_$v -o kt --output-format csv -- \
      python bench.py --workload poisson --no-cpu --steps 100 > gpurun_out/r04_pois_kt_$v.json 2>&1 || exit 1
done
