#!/bin/bash
# Rehearsal of the driver's N = 2/4/8 scaling command at the headline size
# (N = 65536), on a ONE-GPU box: torch.distributed.run with one process per
# rank, exactly as the driver launches bench.py, except that every rank drives
# device 0 with its own NCCL_HOSTID (tests/_bench_rank_wrapper.py), so RCCL
# carries the exchange over its socket transport instead of xGMI and the ranks
# share one GPU's HBM.  The numbers are therefore NOT scaling numbers; what is
# checked is the flow: every rank generates its 65536/P-row block, the timed
# region runs, one JSON line comes from rank 0, and the true residual after
# the fixed-count run is the single-GPU run's.
#   gpurun -- 'bash tools/scale_rehearsal.sh' (prints the per-phase maxima and the RCCL identity)
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/scale_rehearsal
mkdir -p $OUT
port=29631
for P in 2 4 8; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P \
        --master-addr 127.0.0.1 --master-port $((port + P)) \
        tests/_bench_rank_wrapper.py --gpus $P --steps 10 --warmup 2 \
        > $OUT/bench_g$P.json 2> $OUT/bench_g$P.err
    python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/bench_g$P.json') if l.startswith('{')][0]; print($P, round(d['value'],2), d['phases_us']['max_over_ranks'], round(d['phases_us']['tiling_mean_sum_over_ms_per_step'],4), d['rccl']['nranks'], d['rccl']['distinct_devices'])"
done
