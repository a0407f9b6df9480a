#!/bin/bash
# GPU box, round 3: the whole -m gpu suite (one process), configs[4] kernel stats, train-bench A/B of the
# weight-gradient split, weight-gradient SQ / HBM counters.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/rd"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$ROOT/gpurun_out/rd/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$ROOT/gpurun_out/rd/gputests.log" | tail -15
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash "$ROOT/tools/prof_gset.sh" > "$ROOT/gpurun_out/rd/gset_stats.txt" 2>&1 || exit 4
head -8 "$ROOT/gpurun_out/rd/gset_stats.txt" | cut -c1-120
for v in rows even rows2; do
  case $v in rows|rows2) e="";; even) e="ECO_WGRAD_EVEN=1";; esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/rd/b_$v.json" 2>"$ROOT/gpurun_out/rd/b_$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/rd/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
bash "$ROOT/tools/pmc_wgrad.sh" > "$ROOT/gpurun_out/rd/pmc_wgrad.txt" 2>&1 || { tail -5 "$ROOT/gpurun_out/rd/pmc_wgrad.txt"; exit 6; }
tail -4 "$ROOT/gpurun_out/rd/pmc_wgrad.txt" | cut -c1-400
