#!/bin/bash
# GPU box: the whole -m gpu suite on the default library, then the train bench interleaved over library builds.
# usage: bash tools/r04/suite_ab.sh <tag> <lib|default> ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|benched recipe" "$OUT/gputests.log" | tail -8
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    if [ "$lib" != default ]; then export ECO_HIP_LIB=$ROOT/$lib; else unset ECO_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/b${rep}_v$i.json" 2> "$OUT/b${rep}_v$i.err" || { tail -5 "$OUT/b${rep}_v$i.err"; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, round(d['roofline']['avg_launch_ms'],4), d.get('untimed_per_episode_costs',{}).get('evaluate_agent_ms'))" "$OUT/b${rep}_v$i.json" "$lib"
    i=$((i+1))
  done
done
