#!/bin/bash
# A/B of library builds on the train bench: rocprofv3 kernel stats per variant.
# usage: [BENCH_ARGS="--workload gset"] bash tools/ab_lib.sh <tag> <lib.so|default> ...   (GPU box, via gpurun)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  if [ "$lib" != default ]; then export ECO_HIP_LIB=$ROOT/$lib; else unset ECO_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/v$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_v$i.json"
  echo "v$i $lib: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" "$OUT/bench_v$i.json")"
  i=$((i+1))
done
echo done
