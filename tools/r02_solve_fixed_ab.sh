#!/bin/bash
# fp64 solve time at N = 512 / 2048 / 8192: the tree before folding the
# Ap clear and the convergence-record reset into k_residual_f64 (a git
# worktree at _ab_old, built in place) against the current tree, interleaved.
set -euo pipefail
OUT=$PWD/gpurun_out/solve_fixed_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
    for tree in _ab_old .; do
        (cd $tree && timeout -k 10 120 python $OLDPWD/tools/r02_solve_fixed_ab.py 512 2048 8192) >> $OUT
    done
done
cat $OUT
