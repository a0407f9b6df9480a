#!/bin/bash
# PMC passes over the configs[4] bench (gset), each counter set in its own rocprofv3 run: HBM bytes
# (FETCH_SIZE, WRITE_SIZE), L2 hits, LDS bank conflicts / issue, SQ wait counters.  Summarised per kernel
# into gpurun_out/pmc_gset/summary.json (tools/pmc_gset_summary.py).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_gset
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for CS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
          "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD" \
          "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --workload gset --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 "$ROOT/tools/pmc_gset_summary.py" "$OUT"
