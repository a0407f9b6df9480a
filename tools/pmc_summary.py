"""Summarise the tools/run_profile.sh passes into profiles/<round>/<tag>/ (kernel stats + HBM bytes per launch).

usage: python3 tools/pmc_summary.py gpurun_out/prof_<tag> profiles/r01/<tag>

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB = 1024 B), from separate --pmc passes:
MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE counts half of wide streaming reads.  Launches are keyed by
(kernel name, number of workgroups), so the batch-size variants of one kernel stay apart."""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    return name.split("(")[0].split("<")[0].replace("void ", "").replace("eco::", "").strip()


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench_trace.json"), os.path.join(dst, "bench_under_rocprof.json"))
    per = {}
    for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        agg = collections.defaultdict(lambda: [0, 0.0])
        with open(os.path.join(src, sub, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                g = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
                a = agg[(short(r["Kernel_Name"]), g)]
                a[0] += 1
                a[1] += float(r["Counter_Value"])
        for (k, g), (n, v) in agg.items():
            e = per.setdefault(k, {}).setdefault(str(g), {})
            e[ctr + "_KB_per_launch"] = v / n
            e["launches_" + ctr] = n
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, tools/run_profile.sh "
                     f"({os.path.basename(src)}); HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB = 1024 B)",
           "kernels": {}}
    for k, grids in per.items():
        for g, v in grids.items():
            if "FETCH_SIZE_KB_per_launch" in v and "WRITE_SIZE_KB_per_launch" in v:
                b = (2 * v["FETCH_SIZE_KB_per_launch"] + v["WRITE_SIZE_KB_per_launch"]) * 1024
                out["kernels"].setdefault(k, {})[g] = dict(v, hbm_bytes_per_launch=b)
    with open(os.path.join(dst, "pmc_hbm.json"), "w") as f:
        json.dump(out, f, indent=1)
    for k in sorted(out["kernels"]):
        if k.startswith(("mpnn", "wgrad", "env", "act")):
            for g, v in out["kernels"][k].items():
                print(f"{k:40s} blocks {g:>6s}  {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
