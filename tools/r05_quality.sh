#!/bin/bash
# GPU box: tools/r05/quality_sweep.py for one graph family (JSON lines into gpurun_out/<tag>/sweep_<family>.jsonl)
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"; shift
FAM=$1; shift
mkdir -p "$OUT"
timeout -k 10 ${QTIMEOUT:-1100} python -u tools/r05/quality_sweep.py $FAM "$@" > "$OUT/sweep_$FAM.jsonl" 2> "$OUT/sweep_$FAM.err"
rc=$?; cat "$OUT/sweep_$FAM.jsonl"; [ $rc -ne 0 ] && tail -5 "$OUT/sweep_$FAM.err"; exit $rc
