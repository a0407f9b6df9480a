#!/bin/bash
# GPU box: full -m gpu suite, then the train bench twice, phase timing
# of the dense kernels, configs[4] kernel stats.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/wm"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$ROOT/gpurun_out/wm/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$ROOT/gpurun_out/wm/gputests.log" | tail -15
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for v in base base2; do
  e=""
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/wm/b_$v.json" 2>"$ROOT/gpurun_out/wm/b_$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/wm/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
timeout -k 10 300 python -u tools/phase_timing.py > "$ROOT/gpurun_out/wm/phase_er200.txt" 2>&1 || exit 6
head -30 "$ROOT/gpurun_out/wm/phase_er200.txt"
bash "$ROOT/tools/prof_gset.sh" > "$ROOT/gpurun_out/wm/gset_stats.txt" 2>&1 || exit 7
head -9 "$ROOT/gpurun_out/wm/gset_stats.txt" | cut -c1-100
