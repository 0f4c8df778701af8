set -u
D=gpurun_out/r03_symw2; mkdir -p $D
for r in 1 2; do
  timeout -k 10 200 python tools/ab_lib.py ab/libcgx_head.so bench.py --workload symmetric --no-cpu --steps 30 > $D/head_r$r.json 2>/dev/null || exit $?
  CGX_SYM_BLOCKS_PER_CU=2 timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/new2_r$r.json 2>/dev/null || exit $?
  CGX_SYM_NT=0 CGX_SYM_BLOCKS_PER_CU=2 timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/new2nt0_r$r.json 2>/dev/null || exit $?
  for v in head new2 new2nt0; do python3 -c "
import json;d=json.load(open('$D/${v}_r$r.json'));print('$v r$r', round(d['value'],1),'it/s', round(d['matvec_gbps'],1),'GB/s')"; done
done
