#!/bin/bash
# round 4, step 20: the symmetric-storage slow-box question, one attempt
# (VERDICT r03 item 5): classify this box by the symmetric rate, then the
# DRAM read requests per TCC instance for k_symv_f64 and, as the control,
# k_matvec_f64 (is the traffic evenly spread over the channels?)
set -u
export TMPDIR=/tmp
D=gpurun_out/r04_symprobe
mkdir -p $D
timeout -k 10 60 rocprofv3 --list-avail > $D/list_avail.txt 2>&1 || true
grep -E "TCC_EA0_RDREQ_DRAM|TCC_EA0_RDREQ_32B|dimension|DIMENSION" $D/list_avail.txt | head -20
timeout -k 10 120 python3 bench.py --workload symmetric --no-cpu --steps 20 > $D/bench_sym.json 2> $D/bench_sym.err || exit $?
timeout -k 10 120 python3 bench.py --no-cpu --steps 10 > $D/bench_dense.json 2> $D/bench_dense.err || exit $?
python3 -c "
import json
for f in ('$D/bench_sym.json','$D/bench_dense.json'):
    d=[json.loads(l) for l in open(f) if l.startswith('{')][0]; print(f, round(d['value'],2))"
for w in symmetric dense; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B -d $D/pmc_$w -o p --output-format csv -- \
      python3 bench.py --workload $w --no-cpu --phases off --steps 3 --warmup 1 > $D/pmc_$w.json 2> $D/pmc_$w.err || exit $?
done
for w in symmetric dense; do f=$(find $D/pmc_$w -name "*counter_collection.csv" | head -1); echo "== $w $f"; head -3 "$f" | cut -c1-400; python3 -c "
import csv,collections
rows=list(csv.DictReader(open('$f')))
print(len(rows), 'rows; columns', list(rows[0].keys()) if rows else None)
"; done
