#!/bin/bash
# Why k_symv_f64 sits at 94 % of its pattern's read ceiling while
# k_matvec_f64 reaches 99 %: occupancy of the memory pipe and wave stalls,
# three --pmc passes per workload (limits: 8 SQ, 4 TCC, 2 TA, 4 TCP).
#   A: TCC_EA0_RDREQ_LEVEL_sum, TCC_EA0_RDREQ_sum, GRBM_GUI_ACTIVE
#   B: SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
#      SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD
#   C: TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_stalls
mkdir -p $D
run() {
  local w=$1 pass=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $D/${w}_$pass -o p --output-format csv -- \
      python3 bench.py --workload $w --no-cpu --phases off --steps 4 --warmup 1 > /dev/null 2> $D/${w}_$pass.err || exit $?
}
for w in dense symmetric; do
  run $w A TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
  run $w B SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD
  run $w C TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum
done
python3 - <<'PY' > $D/summary.json
import csv, glob, json, collections
D = "gpurun_out/r03_stalls"
out = {}
for w in ("dense", "symmetric"):
    k = "k_matvec_f64" if w == "dense" else "k_symv_f64"
    v = collections.defaultdict(list)
    for f in glob.glob(f"{D}/{w}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"] and "reduce" not in r["Kernel_Name"]:
                v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[w] = {c: sum(x) / len(x) for c, x in v.items()}
print(json.dumps(out, indent=1))
PY
cat $D/summary.json
