#!/bin/bash
# GPU box, end of round 6: the whole -m gpu suite, smoke(), the default bench and the configs lines.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r06final}"
mkdir -p "$OUT"
# -s: the quality pins print one line per trained seed (progress every ~30 s into the log)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|single-attempt ratio" "$OUT/gputests.log" | tail -6
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 4; }
tail -1 "$OUT/smoke.log"
