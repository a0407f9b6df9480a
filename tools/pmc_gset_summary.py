"""Summarise tools/pmc_gset.sh passes: per kernel (launches with a grid of the same size kept apart) the
mean of every counter per launch, HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB = 1024 B; gfx950
FETCH_SIZE counts half of wide streaming reads, MI355X_MICROARCH.md 'HBM') and launches per forward.

usage: python3 tools/pmc_gset_summary.py gpurun_out/pmc_gset [profiles/r02/gset_pmc]"""
import collections
import csv
import glob
import json
import os
import sys


def main(src, dst=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("eco::", "").strip()
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    forwards = None
    out = {"source": "rocprofv3 --pmc, one counter set per run (tools/pmc_gset.sh), bench.py --workload gset "
                     "--steps 2 --warmup 1: HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB = 1024 B)", "kernels": {}}
    for k, v in agg.items():
        if "readout" in k and "FETCH_SIZE" in v:
            forwards = len(v["FETCH_SIZE"])
    for k, v in sorted(agg.items()):
        e = {c: sum(x) / len(x) for c, x in v.items()}
        n = len(v.get("FETCH_SIZE", []))
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if forwards:
            e["launches_per_forward"] = n / forwards
        out["kernels"][k] = e
        print(f"{k[:50]:50s} " + " ".join(f"{c}={x:.4g}" for c, x in sorted(e.items())))
    if dst:
        os.makedirs(dst, exist_ok=True)
        with open(os.path.join(dst, "pmc_hbm.json"), "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
