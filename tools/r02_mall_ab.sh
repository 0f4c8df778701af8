set -euo pipefail
for rep in 1 2; do for nt in 8 2; do CGX_MV_NT=$nt timeout -k 10 200 python tools/iter_floor.py 1024 2048 4096 5792 8192 >> gpurun_out/r02_mall_ab.jsonl 2>&1; done; done
