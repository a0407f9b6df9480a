#!/bin/bash
# GPU box: SQ / GRBM counters of the DL kernels (configs[3] shape: BA-500 m=4, M=2048) over tools/phase_timing.py
# with the product library, one rocprofv3 pass per counter group; summarised by tools/pmc_sq_summary.py.
# usage: bash tools/r04/pmc_dl.sh <tag>
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_dl}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export ECO_HIP_LIB=$ROOT/eco-dqn_amd/eco_hip/libecohip.so
i=0
for CS in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES" \
          "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CS --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/tools/phase_timing.py" --graph BA --n 500 --p 4 > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 5; }
done
python3 - "$OUT" > "$OUT/pmc.txt" <<'PY'
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
python3 "$ROOT/tools/pmc_sq_summary.py" "$OUT/pmc.txt" "$OUT/pmc_sq_dl.json"
