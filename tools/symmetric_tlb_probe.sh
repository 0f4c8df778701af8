# round 5: UTCL1 translation counters of k_symv_f64 over six processes (profiles/r05_symprobe_tlb/)
export TMPDIR=/tmp; D=gpurun_out/r05_tlb; mkdir -p $D
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum"
for i in 1 2 3 4 5 6; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $D/p$i -o p --output-format csv -- python3 bench.py --workload symmetric --no-cpu --steps 10 --warmup 2 --settle 0 > $D/p$i.json 2> $D/p$i.err || exit $?
done
python3 - $D <<'PY'
import csv,glob,json,sys,collections,statistics
D=sys.argv[1]
for i in range(1,7):
    d=[json.loads(l) for l in open(f"{D}/p{i}.json") if l.startswith('{')][0]
    agg=collections.defaultdict(list); dur=[]
    for f in glob.glob(f"{D}/p{i}/**/*counter_collection.csv",recursive=True):
        for r in csv.DictReader(open(f)):
            if 'k_symv_f64' in r['Kernel_Name']:
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
                dur.append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
    print(i, round(d['value'],1), {k.replace('TCP_UTCL1_','')[:22]:round(statistics.median(v)) for k,v in agg.items()}, 'us', round(statistics.median(dur),1) if dur else None)
PY
