#!/bin/bash
# GPU box, round 4: the whole -m gpu suite (stop at the first failure), then the default train bench once.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r04}"
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/gputests.log" | tail -8
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2>"$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
tail -c 3000 "$OUT/bench.json"
