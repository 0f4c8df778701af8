#!/bin/bash
# Every bench workload once on the final tree (short runs): dense N=16384,
# symmetric, Poisson m=8192, streamed N=32768 with and without a resident part.
set -euo pipefail
OUT=gpurun_out
timeout -k 10 200 python bench.py --n 16384 --steps 50 --no-cpu > $OUT/v_dense16k.json 2> $OUT/v_dense16k.err
timeout -k 10 200 python bench.py --workload symmetric --steps 20 --no-cpu > $OUT/v_sym.json 2> $OUT/v_sym.err
timeout -k 10 200 python bench.py --workload poisson --steps 50 --no-cpu > $OUT/v_poisson.json 2> $OUT/v_poisson.err
timeout -k 10 200 python bench.py --workload stream --n 32768 --steps 3 --warmup 1 > $OUT/v_stream.json 2> $OUT/v_stream.err
timeout -k 10 200 python bench.py --workload stream --n 32768 --steps 3 --warmup 1 --resident-gb 6 > $OUT/v_stream_res.json 2> $OUT/v_stream_res.err
timeout -k 10 200 python bench.py --workload stream_symmetric --n 32768 --steps 3 --warmup 1 --resident-gb 8 > $OUT/v_stream_sym_res.json 2> $OUT/v_stream_sym_res.err
