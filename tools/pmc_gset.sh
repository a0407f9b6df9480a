#!/bin/bash
# PMC passes over the configs[4] bench (gset): HBM bytes (FETCH_SIZE, WRITE_SIZE in separate passes),
# L2 hit/miss, SQ stall counters; summarised per kernel.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_gset
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for CS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
          "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
          "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $CS --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --workload gset --steps 2 --warmup 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")[-60:]
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in agg.items():
    if "shared" in k or "env_step" in k:
        print(k, " ".join(f"{c}={sum(x)/len(x):.4g}" for c, x in sorted(v.items())))
PY
