#!/bin/bash
# round 4, step 8: the Poisson kernels' access pattern against contiguous
# streaming of the same mix (hbm_strip_mix), 1-, 2- and 4-KiB row chunks per wave
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/hbm_strip_mix tools/microbench/hbm_strip_mix.hip || exit 1
timeout -k 10 180 /tmp/hbm_strip_mix 8192 > gpurun_out/r04_strip_mix.json || exit 1
cat gpurun_out/r04_strip_mix.json
