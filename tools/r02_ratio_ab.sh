#!/bin/bash
# A/B of the cg_ratio change on the Poisson (configs[4]) and dense N=16384
# benches: the tree before it (a git worktree at _ab_old, built in place) and
# the current tree, interleaved, three rounds.
set -euo pipefail
OUT=$PWD/gpurun_out/ratio_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
    for tree in _ab_old .; do
        for args in "--workload poisson --steps 100" "--n 16384 --steps 25"; do
            (cd $tree && timeout -k 10 120 python bench.py $args --warmup 5 --settle 2 --no-cpu) \
                | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({'tree': '$tree', 'args': '$args', 'it_s': d['value'], 'relres': d['check']['relres']}))" >> $OUT
        done
    done
done
cat $OUT
