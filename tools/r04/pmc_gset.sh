#!/bin/bash
# GPU box: SQ counters of the shared-graph kernels (configs[4] bench, 2 steps) per library build.
# usage: bash tools/r04/pmc_gset.sh <tag> <lib|default> ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  if [ "$lib" != default ]; then export ECO_HIP_LIB=$ROOT/$lib; else unset ECO_HIP_LIB; fi
  j=0
  for CS in "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU" \
            "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    j=$((j+1))
    timeout -k 10 300 rocprofv3 --pmc $CS --output-format csv -d "$OUT/v${i}p$j" -o run -- \
      python3 "$ROOT/bench.py" --workload gset --steps 2 --warmup 1 > "$OUT/v${i}p$j.log" 2>&1 || { tail -5 "$OUT/v${i}p$j.log"; exit 5; }
  done
  echo "== $lib"
  python3 - "$OUT" "v$i" <<'PY'
import csv, glob, sys, collections
out, v = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{out}/{v}p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0]
        if "shared_agg" in k or "shared_lin" in k:
            agg[k.split("<")[0] + row["Kernel_Name"].split("(")[0].split("<")[-1][:2]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    print(k, " ".join(f"{c}={sum(x)/len(x):.4g}" for c, x in sorted(d.items())))
PY
  i=$((i+1))
done
