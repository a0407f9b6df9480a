#!/bin/bash
# PMC passes over tools/phase_timing.py (one forward no-save, one forward save, one backward at
# B=2048 ER-200) with the product library; one rocprofv3 pass per counter group.
# usage: bash tools/pmc_probe.sh <tag> "<counters pass 1>" ["<counters pass 2>" ...]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export ECO_HIP_LIB=$ROOT/eco-dqn_amd/eco_hip/libecohip.so
i=0
for CS in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CS --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/tools/phase_timing.py" > "$OUT/p$i.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.OrderedDict()
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-60:]
        agg.setdefault((row["Dispatch_Id"], k), {})[row["Counter_Name"]] = float(row["Counter_Value"])
for (d, k), v in agg.items():
    if "mpnn" in k:
        print(d, k, " ".join(f"{c}={x:.4g}" for c, x in v.items()))
PY
