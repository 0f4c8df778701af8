#!/bin/bash
# CGX_F32_REF solve time (tools/ref_fuse_ab.py: whole solves at EPSILON 1e-6,
# x checked bitwise against the reference) for the tree before folding the
# convergence-record reset into the fp32 residual kernel (git worktree at
# _ab_old, built in place) against the current tree, interleaved.
set -euo pipefail
OUT=$PWD/gpurun_out/ref_resid_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
    for tree in _ab_old .; do
        (cd $tree && timeout -k 10 120 python tools/ref_fuse_ab.py 512 2048 8192) \
            | python -c "import json,sys; [print(json.dumps(dict(json.loads(l), tree='$tree'))) for l in sys.stdin if l.startswith('{')]" >> $OUT
    done
done
cat $OUT
