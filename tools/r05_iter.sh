#!/bin/bash
# GPU box, one iteration: selected -m gpu tests, phase timing per mask, interleaved configs[2] bench per mask.
# usage: bash tools/r05_iter.sh <tag> "<pytest selection>" "<paths values>"
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
for p in $3; do
  timeout -k 10 120 python -u tools/phase_timing.py --paths $p > "$OUT/phase_p$p.txt" 2>&1 || { tail -5 "$OUT/phase_p$p.txt"; exit 4; }
  echo "== phase p$p"; grep -E "forward|backward|layer [0-2] |staging|A:|B:|C:|readout|DQ|sums|per-graph|dh3" "$OUT/phase_p$p.txt" | head -40
done
for rep in 1 2; do
  for p in $3; do
    ECO_BENCH_KERNEL_PATHS=$p timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > "$OUT/bench_p${p}_r$rep.json" 2> "$OUT/bench_p${p}_r$rep.err" || { tail -5 "$OUT/bench_p${p}_r$rep.err"; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), r.get('kernel'), round(r.get('avg_launch_ms',0) or 0,4))" "$OUT/bench_p${p}_r$rep.json" "p$p r$rep"
  done
done
