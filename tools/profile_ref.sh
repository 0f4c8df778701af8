#!/bin/bash
# Kernel times of an fp32-ref (bit-exact) CLI solve on the device-generated
# N-system (GPU box, repo root):  N=8192 bash tools/profile_ref.sh
set -euo pipefail
export TMPDIR=/tmp
N=${N:-8192}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref -o kt --output-format csv -- \
    conjugate_gradient_amd/bin/cg_hip --spd $N --fp32-ref --stats > gpurun_out/ref_run.log 2>&1
grep -E "clock|iterations" gpurun_out/ref_run.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_ref/kt_kernel_stats.csv")):
    print(r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
