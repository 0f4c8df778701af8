#!/bin/bash
# The wrap-spanning pipeline A/B again, by kernel durations: one rank's
# iteration (tools/microbench/rank_iteration, rank P/2) under rocprofv3
# --kernel-trace for the HEAD build and the new one, G = 8 / 4 / 2, two
# rounds, plus untraced wall times over 300 iterations.
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_wrap2
mkdir -p $D
: > $D/wall.jsonl
for r in 1 2; do
  for g in 8 4 2; do
    for b in head new; do
      bin=tools/microbench/rank_iteration; [ $b = head ] && bin=ab/rank_iteration_head
      echo "{\"build\": \"$b\", \"round\": $r, \"line\": $(timeout -k 10 120 $bin $g 300)}" >> $D/wall.jsonl || exit 1
      timeout -k 10 120 rocprofv3 --kernel-trace -d $D/kt_${b}_g${g}_r$r -o kt --output-format csv -- $bin $g 60 \
          > /dev/null 2>&1 || exit $?
    done
  done
done
python3 - <<'PY'
import csv, glob, json, statistics as st
D = "gpurun_out/r03_wrap2"
for l in open(f"{D}/wall.jsonl"):
    d = json.loads(l)
    print("wall", d["build"], d["round"], d["line"]["ranks"], d["line"]["us_per_iteration_without_collectives"])
out = []
for f in sorted(glob.glob(f"{D}/kt_*/**/kt_kernel_trace.csv", recursive=True)):
    tag = f.split("/")[2]
    rows = [r for r in csv.DictReader(open(f)) if "k_matvec_f64" in r["Kernel_Name"]]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows][10:]
    own, rest = st.median(d[0::2]), st.median(d[1::2])
    out.append({"tag": tag, "own_ns": own, "rest_ns": rest})
    print(tag, own, rest)
json.dump(out, open(f"{D}/kt_summary.json", "w"), indent=1)
PY
