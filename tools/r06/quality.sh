#!/bin/bash
# GPU box: quality sweep variants (tools/r06/quality_sweep.py), one JSON line per (variant, seed).
# usage: bash tools/r06/quality.sh <tag> ER|BA <variant> [<variant> ...]
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"
shift
mkdir -p "$OUT"
timeout -k 10 1050 python -u tools/r06/quality_sweep.py "$@" > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
rc=$?
python3 - "$OUT/sweep.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "seed" in d:
        print(d["name"], d["seed"], round(d["best_one"], 4), round(d["best_fifty"], 4), round(d["final_one"], 4), round(d["train_s"], 1))
    else:
        print(l.strip())
PY
[ $rc -ne 0 ] && tail -5 "$OUT/sweep.err"
exit $rc
