#!/bin/bash
# GPU box: shared-graph parity + configs[4] kernel stats (tiles table fix), then train-bench A/B of the
# weight-gradient workgroup split (ECO_WGRAD_BIG) and the box's cgroup CPU quota.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab"
cat /sys/fs/cgroup/cpu.max 2>&1 || true; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  "tests/test_parity_bench_sizes_gpu.py::test_shared_graph_forward_matches_per_episode_and_oracle" \
  tests/test_parity_bench_sizes_gpu.py::test_shared_graph_forward_hub_and_isolated_nodes \
  tests/test_parity_benched_batches_gpu.py > "$ROOT/gpurun_out/ab/shared_tests.log" 2>&1 \
  || { echo "shared tests rc=$?"; tail -30 "$ROOT/gpurun_out/ab/shared_tests.log"; exit 3; }
tail -2 "$ROOT/gpurun_out/ab/shared_tests.log"
bash "$ROOT/tools/prof_gset.sh" || exit 4
for v in def big96 big112 big128 def2; do
  case $v in
    def|def2) e="";; big96) e="ECO_WGRAD_BIG=96";; big112) e="ECO_WGRAD_BIG=112";; big128) e="ECO_WGRAD_BIG=128";;
  esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab/b_$v.json" 2>"$ROOT/gpurun_out/ab/b_$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
