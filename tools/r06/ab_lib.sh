#!/bin/bash
# GPU box: selected -m gpu tests on the product library, then the configs[2] bench alternating between a
# baseline library (ECO_HIP_LIB=eco_hip/libecohip_<base>.so) and the product one, 2 rounds.
# usage: bash tools/r06/ab_lib.sh <tag> "<pytest selection>" <base> "[bench args]"
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"
mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$OUT/tests.log" | tail -6
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
BASE="$ROOT/eco-dqn_amd/eco_hip/libecohip_$3.so"
for rep in 1 2; do
  for v in base prod; do
    if [ $v = base ]; then export ECO_HIP_LIB="$BASE"; else unset ECO_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ${4:-} \
      > "$OUT/bench_${v}_r$rep.json" 2> "$OUT/bench_${v}_r$rep.err" || { tail -5 "$OUT/bench_${v}_r$rep.err"; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; k=d.get('kernels_ms_per_step',{}); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), round(r.get('avg_launch_ms',0) or 0,4), {a: round(b,3) for a,b in k.items()})" "$OUT/bench_${v}_r$rep.json" "$v r$rep"
  done
done
unset ECO_HIP_LIB
