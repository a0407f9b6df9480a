#!/bin/bash
# GPU box: selected -m gpu tests on the product library, then the configs[2] bench under each library build
# (interleaved, ECO_HIP_LIB).  usage: bash tools/r05_libab.sh <tag> "<pytest selection>" "<lib suffixes>" [bench args]
# ("product" = eco_hip/libecohip.so)
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"
mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$OUT/tests.log" | tail -8
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
for rep in 1 2; do
  for v in $3; do
    lib="$ROOT/eco-dqn_amd/eco_hip/libecohip.so"; [ "$v" != product ] && lib="$ROOT/eco-dqn_amd/eco_hip/libecohip_$v.so"
    ECO_HIP_LIB="$lib" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ${4:-} \
      > "$OUT/bench_${v}_r$rep.json" 2> "$OUT/bench_${v}_r$rep.err" || { tail -5 "$OUT/bench_${v}_r$rep.err"; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), r.get('kernel'), round(r.get('avg_launch_ms',0) or 0,4), round(r['frac'],4), {k: round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})" "$OUT/bench_${v}_r$rep.json" "$v r$rep"
  done
done
