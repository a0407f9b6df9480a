#!/bin/bash
# GPU box: rocprofv3 kernel stats of one bench workload per library build.
# usage: bash tools/r04/kstats.sh <tag> "<bench args>" <lib|default> ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; BARGS=$2; shift 2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  if [ "$lib" != default ]; then export ECO_HIP_LIB=$ROOT/$lib; else unset ECO_HIP_LIB; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/v$i" -o run -- \
    python3 "$ROOT/bench.py" $BARGS > "$OUT/v$i.json" 2> "$OUT/v$i.err" || { tail -5 "$OUT/v$i.err"; exit 5; }
  f=$(find "$OUT/v$i" -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; head -8 "$f" | cut -d, -f1-4
  i=$((i+1))
done
