"""Summarise tools/pmc_poisson_stalls.sh's passes: python tools/pmc_poisson_stalls.py DIR
-> DIR/summary.json.

  rates        the bench lines' it/s (Poisson in three processes, dense once);
  per_launch   per pass and kernel: each counter's mean per launch, the median
               duration, and DRAM credit stalls per 1000 TCC cycles;
  strip_mix    hbm_strip_mix's configurations (reads + writes, blocks per CU,
               walk, XCD bands): achieved GB/s and stalls per 1000 TCC cycles,
               read and write passes, medians over each configuration's 8
               launches (1 warm-up + 7 timed, in the order the program runs
               them: hbm_strip_mix.hip main / mix)."""
import collections
import csv
import glob
import json
import re
import statistics
import sys

POINTS = 8192 * 8192  # hbm_strip_mix's grid at m = 8192


def dispatches(pas):
    by = collections.defaultdict(dict)
    for f in glob.glob(f"{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = by[(f, int(r["Dispatch_Id"]))]
            d["name"] = r["Kernel_Name"]
            d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def stall_rate(d):
    st = d.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", d.get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"))
    cyc = d.get("TCC_CYCLE_sum")
    return 1e3 * st / cyc if st is not None and cyc else None


def kernel_key(name):
    k = re.search(r"(k_\w+)", name)
    if not k or not k.group(1).startswith(("k_poisson", "k_matvec")):
        return None
    xm = re.search(r"k_poisson_xr\w*<[^>]*, (\d)>", name)
    return k.group(1) + (f"<XM{xm.group(1)}>" if xm else "")


def per_launch(pas):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dispatches(pas):
        k = kernel_key(d["name"])
        if k is None:
            continue
        for cn, v in d.items():
            if cn != "name":
                agg[k][cn].append(v)
        r = stall_rate(d)
        if r is not None:
            agg[k]["stall_per_kcycle"].append(r)
    out = {}
    for k, cs in agg.items():
        out[k] = {cn: round(statistics.median(v) if cn in ("us", "stall_per_kcycle") else sum(v) / len(v), 3)
                  for cn, v in cs.items()}
        out[k]["us_median"] = out[k].pop("us")
    return out


def strip_labels():
    labels = []
    for nr, nw in ((5, 2), (2, 1)):
        for bpc in (1, 2):
            labels += [(nr, nw, bpc, "contiguous", 0), (nr, nw, bpc, "contiguous_cpl4", 0)]
            for bands in (0, 1):
                labels += [(nr, nw, bpc, w, bands) for w in ("strip512", "strip1024", "strip2048", "strip512_rpi16")]
    return labels


def strip_mix(pas):
    ks = [d for d in dispatches(pas) if "k_strip" in d["name"]]
    labels = strip_labels()
    if len(ks) != 8 * len(labels):
        return {"error": f"{len(ks)} k_strip launches, expected {8 * len(labels)}"}
    out = []
    for i, (nr, nw, bpc, walk, bands) in enumerate(labels):
        g = ks[8 * i:8 * i + 8]
        us = statistics.median(d["us"] for d in g)
        out.append({"reads": nr, "writes": nw, "blocks_per_cu": bpc, "walk": walk, "bands": bands,
                    "GBps": round(POINTS * 8 * (nr + nw) / (us * 1e-6) / 1e9, 1),
                    "stall_per_kcycle": round(statistics.median(stall_rate(d) for d in g), 2)})
    return out


def main(D):
    out = {"rates": {}, "per_launch": {}, "strip_mix": {}}
    for f in sorted(glob.glob(f"{D}/bench_*.json")):
        try:
            d = [json.loads(ln) for ln in open(f) if ln.startswith("{")][0]
            out["rates"][f.rsplit("/", 1)[1][:-5]] = round(d["value"], 2)
        except (IndexError, ValueError):
            pass
    for pas in sorted(glob.glob(f"{D}/rd_*") + glob.glob(f"{D}/wr_*")):
        if pas.endswith((".json", ".err")):
            continue
        name = pas.rsplit("/", 1)[1]
        if name.endswith("_strip"):
            out["strip_mix"][name] = strip_mix(pas)
        else:
            out["per_launch"][name] = per_launch(pas)
    json.dump(out, open(f"{D}/summary.json", "w"), indent=1)
    print(json.dumps(out["rates"]))


if __name__ == "__main__":
    main(sys.argv[1])
