#!/bin/bash
# TA (texture-address / vector-memory address) busy share of the train loop's big kernels: one rocprofv3 pass,
# TA_BUSY_avr and GRBM_GUI_ACTIVE, kernels filtered by name; summary = TA_BUSY_avr / GRBM_GUI_ACTIVE per kernel.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_ta
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --kernel-include-regex "wgrad_bf3|backward_dense2|forward_dense2" \
  --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
  > "$OUT/p1.log" 2>&1 || { echo "pass failed"; tail -5 "$OUT/p1.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("eco::", "").strip()
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(agg.items()):
    c = {n: sum(x) / len(x) for n, x in v.items()}
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    print(f"{k:45s} n={len(v.get('GRBM_GUI_ACTIVE', []))} " + " ".join(f"{n}={x:.4g}" for n, x in sorted(c.items())) +
          (f" ta_avr_share={c.get('TA_BUSY_avr', 0) / g:.3f} ta_max_share={c.get('TA_BUSY_max', 0) / g:.3f}" if g else ""))
PY
