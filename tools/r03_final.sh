#!/bin/bash
# GPU box, round 3 final: the -m gpu suite (stop at the first failure), the train bench twice, dense phase timing,
# then the profiles: train kernel trace + FETCH_SIZE + WRITE_SIZE passes, configs[3]/[4]/[1] under rocprof,
# BA-500 phase timing, dense SQ counters.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/fin"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$ROOT/gpurun_out/fin/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$ROOT/gpurun_out/fin/gputests.log" | tail -8
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for v in b1 b2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/fin/$v.json" 2>"$ROOT/gpurun_out/fin/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/fin/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
timeout -k 10 300 python -u tools/phase_timing.py > "$ROOT/gpurun_out/fin/phase_er200.txt" 2>&1 || exit 6
bash "$ROOT/tools/run_profile.sh" r03final > "$ROOT/gpurun_out/fin/run_profile.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/fin/run_profile.log"; exit 7; }
python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/prof_r03final" "$ROOT/gpurun_out/fin/train" || exit 8
bash "$ROOT/tools/r03_configs.sh" > "$ROOT/gpurun_out/fin/configs.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/fin/configs.log"; exit 9; }
grep -E "^(ba500|gset|er20) " "$ROOT/gpurun_out/fin/configs.log"
bash "$ROOT/tools/pmc_dense.sh" > /dev/null 2>&1 || exit 10
python3 "$ROOT/tools/pmc_sq_summary.py" "$ROOT/gpurun_out/pmc_dense.txt" "$ROOT/gpurun_out/fin/train/pmc_sq_dense.json"
