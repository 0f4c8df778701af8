#!/bin/bash
# The Poisson slow-mode probe (round 4's symmetric probe,
# profiles/r04_symprobe/, applied to configs[4]).  On whatever box this runs:
#   1. the Poisson bench rate in three separate processes (the slow mode
#      showed up bimodally per process on some boxes), and the dense one;
#   2. per process, TCC DRAM read credit stalls, 32-B DRAM read requests and
#      TCC cycles per launch of k_poisson_p_f64 / k_poisson_xr_f64 /
#      k_poisson_xr_pipe_f64, against k_matvec_f64 (which runs at the read
#      ceiling on every box), each pass with its own kernel durations;
#   3. the same for the write side where the counters exist;
#   4. the same two passes over tools/microbench/hbm_strip_mix (the kernels'
#      access pattern without arithmetic, at and below its ceiling), if built.
# tools/pmc_poisson_stalls.py writes $D/summary.json.
# Each rocprofv3 pass is its own run (one TCC counter group each).
#   gpurun -- 'bash tools/pmc_poisson_stalls.sh'   (OUT=gpurun_out/... to relocate)
set -u
export TMPDIR=/tmp
D=${OUT:-gpurun_out/poisson_stalls}
mkdir -p "$D"
timeout -s KILL 60 rocprofv3 -L > "$D/counters.txt" 2>&1 || true
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --workload poisson --no-cpu --steps 100 --warmup 10 --settle 1 \
      > "$D/bench_poisson_$i.json" 2> "$D/bench_poisson_$i.err" || exit $?
done
timeout -k 10 150 python3 bench.py --no-cpu --steps 10 > "$D/bench_dense.json" 2> "$D/bench_dense.err" || exit $?
RD="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_CYCLE_sum"
WR="TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_64B_sum TCC_CYCLE_sum"
for i in 1 2 3; do
  timeout -s KILL 90 rocprofv3 --pmc $RD -d "$D/rd_poisson_$i" -o p --output-format csv -- \
      python3 bench.py --workload poisson --no-cpu --steps 6 --warmup 2 --settle 0 \
      > "$D/rd_poisson_$i.json" 2> "$D/rd_poisson_$i.err" || exit $?
done
timeout -s KILL 90 rocprofv3 --pmc $RD -d "$D/rd_dense" -o p --output-format csv -- \
    python3 bench.py --no-cpu --phases off --steps 3 --warmup 1 --settle 0 > "$D/rd_dense.json" 2> "$D/rd_dense.err" \
    || exit $?
if grep -q "TCC_EA0_WRREQ_DRAM_CREDIT_STALL" "$D/counters.txt"; then
  timeout -s KILL 90 rocprofv3 --pmc $WR -d "$D/wr_poisson" -o p --output-format csv -- \
      python3 bench.py --workload poisson --no-cpu --steps 6 --warmup 2 --settle 0 \
      > "$D/wr_poisson.json" 2> "$D/wr_poisson.err" || exit $?
fi
SM=tools/microbench/bin/hbm_strip_mix  # hipcc --offload-arch=gfx950 -O3 -std=c++17 -o $SM tools/microbench/hbm_strip_mix.hip
if [ -x "$SM" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $RD -d "$D/rd_strip" -o p --output-format csv -- $SM 8192 \
      > "$D/rd_strip.json" 2> "$D/rd_strip.err" || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $WR -d "$D/wr_strip" -o p --output-format csv -- $SM 8192 \
      > "$D/wr_strip.json" 2> "$D/wr_strip.err" || exit $?
fi
python3 tools/pmc_poisson_stalls.py "$D"
