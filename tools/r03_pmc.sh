#!/bin/bash
# GPU box, round 3: shared-graph parity + configs[4] kernel stats and PMC, then the configs[2] train PMC
# (kernel trace, FETCH_SIZE, WRITE_SIZE passes) and the dense kernels' SQ counters.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  "tests/test_parity_bench_sizes_gpu.py::test_shared_graph_forward_matches_per_episode_and_oracle" \
  tests/test_parity_bench_sizes_gpu.py::test_shared_graph_forward_hub_and_isolated_nodes \
  tests/test_parity_benched_batches_gpu.py > "$ROOT/gpurun_out/shared_tests.log" 2>&1 \
  || { echo "shared tests rc=$?"; tail -30 "$ROOT/gpurun_out/shared_tests.log"; exit 3; }
tail -3 "$ROOT/gpurun_out/shared_tests.log"
bash "$ROOT/tools/prof_gset.sh" || exit 4
bash "$ROOT/tools/pmc_gset.sh" > "$ROOT/gpurun_out/pmc_gset.txt" 2>&1 || { tail "$ROOT/gpurun_out/pmc_gset.txt"; exit 5; }
tail -20 "$ROOT/gpurun_out/pmc_gset.txt"
[ "${1:-}" = "gset" ] && exit 0
bash "$ROOT/tools/run_profile.sh" r03train || exit 6
python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/prof_r03train" "$ROOT/gpurun_out/r03train" || exit 7
bash "$ROOT/tools/pmc_dense.sh" > /dev/null 2>&1 || exit 8
python3 "$ROOT/tools/pmc_sq_summary.py" "$ROOT/gpurun_out/pmc_dense.txt" "$ROOT/gpurun_out/r03train/pmc_sq_dense.json"
