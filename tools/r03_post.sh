#!/bin/bash
# GPU box: backward / train-step parity after the readout revert, the train bench twice, train kernel stats.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/post"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_dqn_gpu.py tests/test_parity_bench_sizes_gpu.py tests/test_parallel_gpu.py > "$ROOT/gpurun_out/post/tests.log" 2>&1 \
  || { echo "tests rc=$?"; tail -30 "$ROOT/gpurun_out/post/tests.log"; exit 3; }
tail -2 "$ROOT/gpurun_out/post/tests.log"
for v in b1 b2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/post/$v.json" 2>"$ROOT/gpurun_out/post/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/post/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$ROOT/gpurun_out/post/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$ROOT/gpurun_out/post/bench_trace.json" || exit 6
head -6 "$ROOT/gpurun_out/post/trace/run_kernel_stats.csv" | cut -d, -f1-4
