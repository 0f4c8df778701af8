#!/bin/bash
# The Poisson slow-mode probe (round 4's symmetric probe,
# profiles/r04_symprobe/, applied to configs[4]).  On whatever box this runs:
#   1. the Poisson bench rate in three separate processes (the slow mode
#      showed up bimodally per process on some boxes), and the dense one;
#   2. per process, TCC DRAM read credit stalls, 32-B DRAM read requests and
#      TCC cycles per launch of k_poisson_p_f64 / k_poisson_xr_f64 /
#      k_poisson_xr_pipe_f64, against k_matvec_f64 (which runs at the read
#      ceiling on every box), each pass with its own kernel durations;
#   3. the same for the write side where the counters exist.
# Each rocprofv3 pass is its own run (one TCC counter group each).
#   gpurun -- 'bash tools/pmc_poisson_stalls.sh'   (OUT=gpurun_out/... to relocate)
set -u
export TMPDIR=/tmp
D=${OUT:-gpurun_out/poisson_stalls}
mkdir -p "$D"
timeout -s KILL 60 rocprofv3 -L > "$D/counters.txt" 2>&1 || true
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --workload poisson --no-cpu --steps 100 --warmup 10 --settle 1 \
      > "$D/bench_poisson_$i.json" 2> "$D/bench_poisson_$i.err" || exit $?
done
timeout -k 10 150 python3 bench.py --no-cpu --steps 10 > "$D/bench_dense.json" 2> "$D/bench_dense.err" || exit $?
RD="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_CYCLE_sum"
WR="TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_64B_sum TCC_CYCLE_sum"
for i in 1 2 3; do
  timeout -s KILL 90 rocprofv3 --pmc $RD -d "$D/rd_poisson_$i" -o p --output-format csv -- \
      python3 bench.py --workload poisson --no-cpu --steps 6 --warmup 2 --settle 0 \
      > "$D/rd_poisson_$i.json" 2> "$D/rd_poisson_$i.err" || exit $?
done
timeout -s KILL 90 rocprofv3 --pmc $RD -d "$D/rd_dense" -o p --output-format csv -- \
    python3 bench.py --no-cpu --phases off --steps 3 --warmup 1 --settle 0 > "$D/rd_dense.json" 2> "$D/rd_dense.err" \
    || exit $?
if grep -q "TCC_EA0_WRREQ_DRAM_CREDIT_STALL" "$D/counters.txt"; then
  timeout -s KILL 90 rocprofv3 --pmc $WR -d "$D/wr_poisson" -o p --output-format csv -- \
      python3 bench.py --workload poisson --no-cpu --steps 6 --warmup 2 --settle 0 \
      > "$D/wr_poisson.json" 2> "$D/wr_poisson.err" || exit $?
fi
python3 - "$D" <<'PY'
import collections, csv, glob, json, re, sys
D = sys.argv[1]
out = {"rates": {}, "per_launch": {}}
for f in sorted(glob.glob(f"{D}/bench_*.json")):
    try:
        d = [json.loads(l) for l in open(f) if l.startswith("{")][0]
        out["rates"][f.rsplit("/", 1)[1][:-5]] = round(d["value"], 2)
    except (IndexError, ValueError):
        pass
for pas in sorted(glob.glob(f"{D}/rd_*") + glob.glob(f"{D}/wr_*")):
    if pas.endswith((".json", ".err")):
        continue
    agg = collections.defaultdict(list)
    dur = collections.defaultdict(set)
    for f in glob.glob(f"{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.search(r"(k_\w+)", r["Kernel_Name"])
            if not k or not k.group(1).startswith(("k_poisson", "k_matvec")):
                continue
            name = k.group(1) + ("<XM3>" if "k_poisson_xr" in k.group(1) and ", 3>" in r["Kernel_Name"] else
                                 "<XM0>" if "k_poisson_xr" in k.group(1) and ", 0>" in r["Kernel_Name"] else "")
            agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
            dur[name].add((r["Dispatch_Id"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    res = {}
    for (k, cn), v in sorted(agg.items()):
        res.setdefault(k, {})[cn] = round(sum(v) / len(v))
    for k, s in dur.items():
        res.setdefault(k, {})["us_median"] = round(sorted(d for _, d in s)[len(s) // 2], 1)
        cyc = res[k].get("TCC_CYCLE_sum")
        st = res[k].get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", res[k].get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"))
        if cyc and st is not None:
            res[k]["stall_per_kcycle"] = round(1e3 * st / cyc, 3)
    out["per_launch"][pas.rsplit("/", 1)[1]] = res
json.dump(out, open(f"{D}/summary.json", "w"), indent=1)
print(json.dumps(out["rates"]))
PY
