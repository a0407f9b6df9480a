#!/bin/bash
# GPU box: the dense / DQN train-step parity tests after the per-call max-degree reuse and the TD zero-fill
# fusion, then two train-bench lines.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/td"
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_dqn_gpu.py tests/test_parity_bench_sizes_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$ROOT/gpurun_out/td/tests.log" 2>&1
rc=$?; tail -3 "$ROOT/gpurun_out/td/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in b1 b2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/td/$v.json" 2>"$ROOT/gpurun_out/td/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/td/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3))"
done
