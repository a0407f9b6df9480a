#!/bin/bash
# GPU box, one iteration: selected -m gpu tests in one process, then bench lines (each under its own limit).
# usage: bash tools/r06/iter.sh <tag> "<pytest selection>" "<bench args; bench args; ...>"
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"
mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest $2 -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$OUT/tests.log" | tail -8
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
i=0
IFS=';' read -ra BENCHES <<< "${3:-}"
for b in "${BENCHES[@]}"; do
  [ -z "${b// }" ] && continue
  i=$((i+1))
  timeout -k 10 400 python -u bench.py $b > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || { echo "bench $i failed"; tail -20 "$OUT/bench_$i.err"; exit 5; }
  python3 - "$OUT/bench_$i.json" "$b" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
u = d.get("untimed_per_episode_costs") or {}
l = d.get("learn_loop") or {}
print(sys.argv[2], "|", round(d["value"]), round(d["ms_per_step"], 3), r.get("kernel"), round(r.get("avg_launch_ms", 0) or 0, 4),
      round(r["frac"], 4), "| eval ov", round(u.get("evaluate_overlapped_ms", -1), 2), "sync", round(u.get("evaluate_agent_ms", -1), 2),
      "eager", round(u.get("evaluate_agent_eager_launches_ms", -1), 2), "amort", round(u.get("amortised_ms_per_vector_step", -1), 3),
      "| learn", round(l.get("value", -1)), round(l.get("ratio_to_headline", -1), 3), l.get("evaluations"))
PY
done
