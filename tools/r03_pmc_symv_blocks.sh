#!/bin/bash
# k_symv_f64 with one vs two 256-thread blocks per CU: DRAM reads in flight
# and their latency (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ), next to the bench.
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_symblk
mkdir -p $D
for b in 1 2; do
  CGX_SYM_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --workload symmetric --no-cpu --steps 30 > $D/bench_b$b.json 2>/dev/null || exit $?
  CGX_SYM_BLOCKS_PER_CU=$b timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE \
      -d $D/pmc_b$b -o p --output-format csv -- python3 bench.py --workload symmetric --no-cpu --phases off --steps 4 --warmup 1 \
      > /dev/null 2> $D/pmc_b$b.err || exit $?
done
python3 - <<'PY'
import csv, glob, json, collections
D = "gpurun_out/r03_symblk"
for b in (1, 2):
    d = json.load(open(f"{D}/bench_b{b}.json"))
    v = collections.defaultdict(list)
    for f in glob.glob(f"{D}/pmc_b{b}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_symv_f64" in r["Kernel_Name"]:
                v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {c: sum(x) / len(x) for c, x in v.items()}
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    print(json.dumps({"blocks_per_cu": b, "it_s": d["value"], "GBps": d["matvec_gbps"],
                      "reads_in_flight": m["TCC_EA0_RDREQ_LEVEL_sum"] / cyc,
                      "latency_cycles": m["TCC_EA0_RDREQ_LEVEL_sum"] / m["TCC_EA0_RDREQ_sum"]}))
PY
