#!/bin/bash
# Per-rank HBM traffic of the P = 2/4/8 matVec (own block + rest) on the final
# round-2 kernels: two separate --pmc passes per P (tools/pmc_shards.py run),
# each under its own time limit; summarised on the CPU side afterwards with
#   python tools/pmc_shards.py summarise --n 65536 --shards P --tag r02 \
#       --fetch gpurun_out/pmc_g<P>_f/f_counter_collection.csv \
#       --write gpurun_out/pmc_g<P>_w/w_counter_collection.csv
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out
for P in 2 4 8; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_g${P}_f -o f --output-format csv -- \
        python tools/pmc_shards.py run --n 65536 --shards $P > $OUT/pmc_g${P}_f.log 2>&1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_g${P}_w -o w --output-format csv -- \
        python tools/pmc_shards.py run --n 65536 --shards $P > $OUT/pmc_g${P}_w.log 2>&1
    echo "P=$P done"
done
