#!/bin/bash
# GPU box: env-step parity tests, the per-phase wall-clock stamps (timing build) and the envstep sub-bench.
# usage: bash tools/r05_env.sh <tag> [pytest selection]
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r05_env}"
SEL=${2:-"tests/test_env_gpu.py tests/test_problems_gpu.py tests/test_large_gpu.py"}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > "$OUT/tests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/tests.log" | tail -5
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -u tools/r04/env_timing.py > "$OUT/env_timing.log" 2>&1 || { tail -5 "$OUT/env_timing.log"; exit 5; }
cat "$OUT/env_timing.log"
timeout -k 10 200 python -u bench.py --workload envstep --steps 200 --warmup 20 > "$OUT/envstep.json" 2> "$OUT/envstep.err" || { tail -5 "$OUT/envstep.err"; exit 6; }
tail -c 900 "$OUT/envstep.json"; echo
