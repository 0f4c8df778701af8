#!/bin/bash
# Poisson configs[4]: rows per work item (CGX_STENCIL_ROWS) and the halo-row
# load policy (CGX_STENCIL_HALO_T) against it/s and the calibrated DRAM bytes
# of both kernels (TCC_EA0_RDREQ_DRAM_32B / WRREQ_WRITE_DRAM_32B, x32 B).
set -u
export TMPDIR=/tmp
D=gpurun_out/r03_prows
mkdir -p $D
for cfg in "8 1" "16 1" "32 1" "8 0" "16 0"; do
  set -- $cfg
  tag=rows$1_ht$2
  CGX_STENCIL_ROWS=$1 CGX_STENCIL_HALO_T=$2 timeout -k 10 200 python bench.py --workload poisson --no-cpu --steps 200 \
      > $D/$tag.json 2> $D/$tag.err || exit $?
  CGX_STENCIL_ROWS=$1 CGX_STENCIL_HALO_T=$2 timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum \
      TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_64B_sum -d $D/pmc_$tag -o p --output-format csv -- \
      python3 bench.py --workload poisson --no-cpu --steps 4 --warmup 1 > /dev/null 2> $D/pmc_$tag.err || exit $?
  python3 - "$D" "$tag" <<'PY'
import csv, glob, json, sys, collections
d, tag = sys.argv[1], sys.argv[2]
b = json.load(open(f"{d}/{tag}.json"))
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/pmc_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "poisson" in k:
            v["p" if "poisson_p" in k else "xr"][r["Counter_Name"]].append(float(r["Counter_Value"]))
pts = 8192 * 8192
out = {"tag": tag, "it_s": b["value"]}
for k, cs in v.items():
    m = {c: sum(x) / len(x) for c, x in cs.items()}
    out[k] = {"rd_B_pt": 32 * m["TCC_EA0_RDREQ_DRAM_32B_sum"] / pts, "wr_B_pt": 32 * m["TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"] / pts,
              "rd64_B_pt": 64 * m["TCC_EA0_RDREQ_64B_sum"] / pts, "launches": len(cs["TCC_EA0_RDREQ_DRAM_32B_sum"])}
print(json.dumps(out))
PY
done
