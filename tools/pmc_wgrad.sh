#!/bin/bash
# SQ / TA counters of the weight-gradient and backward kernels inside the configs[2] train bench (two short
# bench runs per counter set, kernels filtered by name); one rocprofv3 pass per counter group.
# usage: bash tools/pmc_wgrad.sh [regex]
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
RX=${1:-wgrad_bf3|backward_dense2}
OUT=$ROOT/gpurun_out/pmc_wgrad
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for CS in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES" \
          "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
          "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CS --kernel-include-regex "$RX" --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("eco::", "").strip()
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for k, v in agg.items():
    c = {n: sum(x) / len(x) for n, x in v.items()}
    if "GRBM_GUI_ACTIVE" in c:
        c["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
        c["wait_any_share"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        c["active_share"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        c["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    res[k] = c
    print(k, " ".join(f"{n}={x:.4g}" for n, x in sorted(c.items())))
json.dump({"source": "tools/pmc_wgrad.sh: rocprofv3 --pmc per counter set over bench.py --steps 2 --warmup 1, "
           "kernels filtered by name; HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB = 1024 B)", "kernels": res},
          open(out + "/summary.json", "w"), indent=1)
PY
