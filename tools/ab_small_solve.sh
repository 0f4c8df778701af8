#!/bin/bash
# Interleaved A/B of whole-solve latency at the reference's sizes (GPU box, repo root):
# tools/small_solve_trace.py against two builds of libcgx.so, fp32-ref (flags 1) and fp64 (0).
#   cp conjugate_gradient_amd/lib/libcgx.so ab/libcgx_base.so   # before the change, then rebuild
#   BASE=ab/libcgx_base.so ROUNDS=3 SIZES=512,2048,8192 bash tools/ab_small_solve.sh > profiles/rNN_x_ab.jsonl
# Or an environment knob on one build: VAR=CGX_LOOKAHEAD VALUES="2 1" bash tools/ab_small_solve.sh
set -euo pipefail
export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-3}); do
  if [ -n "${VAR:-}" ]; then
    for v in ${VALUES:-0 1}; do
      for fl in ${FLAGS:-1 0}; do
        env "$VAR=$v" CGX_SMALL_FLAGS=$fl timeout -k 10 120 python tools/small_solve_trace.py ${SIZES:-512,1024,2048,4096,8192} 20 |
          sed "s/^{/{\"round\": $round, \"$VAR\": \"$v\", /"
      done
    done
  else
    for lib in "${BASE:?BASE=<baseline libcgx.so>}" conjugate_gradient_amd/lib/libcgx.so; do
      for fl in ${FLAGS:-1 0}; do
        CGX_AB_LIB=$PWD/$lib CGX_SMALL_FLAGS=$fl timeout -k 10 120 python tools/small_solve_trace.py \
          ${SIZES:-512,1024,2048,4096,8192} 20 | sed "s/^{/{\"round\": $round, /"
      done
    done
  fi
done
