#!/bin/bash
# GPU box, end of round 5: the whole -m gpu suite, smoke(), the default bench and the configs lines.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r05final}"
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gputests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/gputests.log" | tail -5
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 4; }
tail -1 "$OUT/smoke.log"
for w in train er20 gset ba500; do
  case $w in
    train) args="";;
    er20) args="--workload er20 --steps 40 --warmup 5";;
    gset) args="--workload gset --steps 20 --warmup 3";;
    ba500) args="--graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline";;
  esac
  timeout -k 10 400 python -u bench.py $args > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 5; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],4), d.get('launch','')[:20], round(d['roofline']['frac'],4))" "$OUT/bench_$w.json" $w
done
