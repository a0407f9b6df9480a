#!/bin/bash
# GPU box: the -m gpu suite, then the configs[2] and configs[3] bench lines (each under its own time limit).
# usage: bash tools/r05_base.sh <tag> [pytest selection]
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r05}"
SEL=${2:-tests}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/gputests.log" | tail -5
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$OUT/er200.json" 2> "$OUT/er200.err" || { tail -5 "$OUT/er200.err"; exit 5; }
tail -c 400 "$OUT/er200.json"; echo
timeout -k 10 400 python -u bench.py --graph BA --n 500 --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/ba500.json" 2> "$OUT/ba500.err" || { tail -5 "$OUT/ba500.err"; exit 6; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ba500', round(d['value']), round(d['ms_per_step'],3))" "$OUT/ba500.json"
