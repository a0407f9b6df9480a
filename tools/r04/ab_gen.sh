#!/bin/bash
# GPU box: parity tests on the default library, then one bench workload interleaved over library builds.
# usage: bash tools/r04/ab_gen.sh <tag> "<test files>" "<bench args>" <lib|default> ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TESTS=$2; BARGS=$3; shift 3
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$OUT/tests.log" | tail -8
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    if [ "$lib" != default ]; then export ECO_HIP_LIB=$ROOT/$lib; else unset ECO_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py $BARGS > "$OUT/b${rep}_v$i.json" 2> "$OUT/b${rep}_v$i.err" || { tail -5 "$OUT/b${rep}_v$i.err"; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],4), d.get('kernels_ms_per_step'))" "$OUT/b${rep}_v$i.json" "$lib"
    i=$((i+1))
  done
done
