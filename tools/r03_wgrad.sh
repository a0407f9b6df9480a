#!/bin/bash
# GPU box: fp16x2 weight-gradient reduction -- backward / train_step / bench-size parity, then bench A/B against
# the bf16x3 kernel and workgroup counts, then (arg "pmc") the round-3 PMC passes of tools/r03_pmc.sh.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/wg"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_dqn_gpu.py tests/test_parity_bench_sizes_gpu.py tests/test_parity_benched_batches_gpu.py \
  > "$ROOT/gpurun_out/wg/tests.log" 2>&1 || { echo "tests rc=$?"; tail -40 "$ROOT/gpurun_out/wg/tests.log"; exit 3; }
tail -3 "$ROOT/gpurun_out/wg/tests.log"
for v in fh bf3 fh2 fh4; do
  case $v in
    fh) e="";; bf3) e="ECO_WGRAD_BF3=1";; fh2) e="ECO_WGRAD_WG_X=2";; fh4) e="ECO_WGRAD_WG_X=4";;
  esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/wg/b_$v.json" 2>&1 || exit 4
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/wg/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
if [ "${1:-}" = "pmc" ]; then bash "$ROOT/tools/r03_pmc.sh"; exit $?; fi
exit 0
