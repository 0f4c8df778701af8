#!/bin/bash
# round 4, step 21: the symmetric slow-box attempt, continued on whatever box
# comes: the rates, then per-channel DRAM read requests (rocpd database
# output, which may keep the 16 x 8 TCC instances apart) and DRAM credit
# stalls for k_symv_f64 against k_matvec_f64
set -u
export TMPDIR=/tmp
D=gpurun_out/r04_symprobe2
mkdir -p $D
timeout -k 10 120 python3 bench.py --workload symmetric --no-cpu --steps 20 > $D/bench_sym.json 2> $D/bench_sym.err || exit $?
timeout -k 10 120 python3 bench.py --no-cpu --steps 10 > $D/bench_dense.json 2> $D/bench_dense.err || exit $?
python3 -c "
import json
for f in ('$D/bench_sym.json','$D/bench_dense.json'):
    d=[json.loads(l) for l in open(f) if l.startswith('{')][0]; print(f, round(d['value'],2))"
for w in symmetric dense; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B -d $D/db_$w -o p -- \
      python3 bench.py --workload $w --no-cpu --phases off --steps 3 --warmup 1 > $D/db_$w.json 2> $D/db_$w.err || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_CYCLE_sum -d $D/st_$w -o p \
      --output-format csv -- python3 bench.py --workload $w --no-cpu --phases off --steps 3 --warmup 1 > $D/st_$w.json 2> $D/st_$w.err || exit $?
done
python3 - <<PY
import sqlite3, glob, re, collections, csv
for w in ("symmetric", "dense"):
    for f in glob.glob("$D/db_%s/**/*.db" % w, recursive=True):
        c = sqlite3.connect(f)
        tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
        print(w, f, [t for t in tabs if 'pmc' in t.lower() or 'counter' in t.lower()][:12])
        for t in tabs:
            if re.match(r'rocpd_pmc_event$', t) or t == 'pmc_events':
                cols = [r[1] for r in c.execute("pragma table_info(%s)" % t)]
                print(' ', t, cols)
                for r in c.execute("select * from %s limit 3" % t): print('   ', r)
    for f in glob.glob("$D/st_%s/**/*counter_collection.csv" % w, recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = re.search(r'(k_\w+)', r['Kernel_Name'])
            if k and k.group(1) in ('k_symv_f64', 'k_matvec_f64'):
                agg[(k.group(1), r['Counter_Name'])].append(float(r['Counter_Value']))
        for (k, cn), v in sorted(agg.items()): print(w, k, cn, round(sum(v) / len(v)))
PY
