#!/bin/bash
# GPU box: phase timing (timing build) and rocprofv3 kernel stats of the configs[2] bench per kernel-path mask.
# usage: bash tools/r05_prof.sh <tag> "<paths values>" [bench args]
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"
mkdir -p "$OUT"
for p in $2; do
  timeout -k 10 120 python -u tools/phase_timing.py --paths $p > "$OUT/phase_p$p.txt" 2>&1 || { tail -5 "$OUT/phase_p$p.txt"; exit 4; }
  echo "== phase p$p"; grep -E "forward|backward|layer|staging|A:|B:|C:|readout" "$OUT/phase_p$p.txt" | head -40
done
cd /tmp && export TMPDIR=/tmp
for p in $2; do
  ECO_BENCH_KERNEL_PATHS=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_p$p" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ${3:-} > "$OUT/bench_prof_p$p.json" 2> "$OUT/bench_prof_p$p.err" \
    || { tail -5 "$OUT/bench_prof_p$p.err"; exit 5; }
  f=$(find "$OUT/prof_p$p" -name "*kernel_stats.csv" | head -1)
  echo "== stats p$p"; head -12 "$f" | cut -d, -f1-8
done
