#!/bin/bash
# Is the symmetric matVec clock- or power-bound on this box?  Sample the GPU's
# power and clocks every ~0.5 s while the symmetric bench runs, then while the
# dense bench runs (rocm-smi in the background, killed by PID afterwards).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
sample() {  # tag
  ( while true; do echo "T $(date +%s.%N)"; timeout 5 rocm-smi --showpower --showclocks --showtemp 2>&1 \
      | grep -E "Power|sclk|mclk|fclk|Temperature" ; sleep 0.3; done ) > gpurun_out/r03_clk_$1.txt 2>&1 &
  SPID=$!
}
sample sym
timeout -k 10 240 python bench.py --workload symmetric --no-cpu --steps 2000 --warmup 3 > gpurun_out/r03_clk_sym.json
rc=$?
kill $SPID; wait $SPID 2>/dev/null
[ $rc -eq 0 ] || exit $rc
sample dense
timeout -k 10 240 python bench.py --no-cpu --steps 300 --warmup 3 > gpurun_out/r03_clk_dense.json
rc=$?
kill $SPID; wait $SPID 2>/dev/null
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json
for t in ('sym','dense'):
    d=json.load(open('gpurun_out/r03_clk_%s.json'%t)); print(t, round(d['value'],1), round(d['roofline']['achieved'],1))"
for t in sym dense; do echo "== $t"; grep -E "Power|sclk|mclk|fclk" gpurun_out/r03_clk_$t.txt | sort | uniq -c | sort -rn | head -12; done
