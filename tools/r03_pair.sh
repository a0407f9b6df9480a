#!/bin/bash
# GPU box: the paired s' forward -- parity (pair vs two forwards, DQN train-step tests), then train-bench A/B
# (ECO_MPNN_NO_PAIR = two launches) interleaved.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/pair"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_dense_gpu.py tests/test_dqn_gpu.py tests/test_parity_bench_sizes_gpu.py::test_learn_er200_first_train_step_matches_oracle \
  tests/test_parallel_gpu.py > "$ROOT/gpurun_out/pair/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$ROOT/gpurun_out/pair/tests.log"; exit 3; }
tail -2 "$ROOT/gpurun_out/pair/tests.log"
for v in pair nopair pair2 nopair2; do
  case $v in pair|pair2) e="";; nopair|nopair2) e="ECO_MPNN_NO_PAIR=1";; esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/pair/$v.json" 2>"$ROOT/gpurun_out/pair/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/pair/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
