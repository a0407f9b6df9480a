#!/bin/bash
# GPU box, round 4: the tests added this round (one process), the ER-200 benched-recipe quality pin, then the bench.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r04n}"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_kernel_paths_gpu.py tests/test_graph_id_bounds_gpu.py \
  tests/test_dqn_gpu.py tests/test_parity_bench_sizes_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/new_tests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/new_tests.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_training_quality_er200_gpu.py -m gpu -v -s --timeout 380 \
  --timeout-method thread -p no:cacheprovider > "$OUT/quality_er200.log" 2>&1
qrc=$?
grep -E "benched recipe|FAILED|passed|failed" "$OUT/quality_er200.log" | tail -4
if [ $qrc -ne 0 ] && [ $qrc -ne 1 ]; then echo "quality rc=$qrc: stopping"; exit $qrc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2>"$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
tail -c 4000 "$OUT/bench.json"
exit $(( rc > qrc ? rc : qrc ))
