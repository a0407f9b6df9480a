#!/bin/bash
# GPU box: the default bench line (configs[2], with the CPU baseline) and the configs[1] / [4] / [3] lines.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r06bench}"
mkdir -p "$OUT"
for w in train er20 gset ba500; do
  case $w in
    train) args="--steps 20 --warmup 5";;
    er20) args="--workload er20 --steps 40 --warmup 5";;
    gset) args="--workload gset --steps 20 --warmup 3";;
    ba500) args="--graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline";;
  esac
  timeout -k 10 400 python -u bench.py $args > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 5; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); l=d.get('learn_loop') or {}; print(sys.argv[2], round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), round(l.get('value',0)))" "$OUT/bench_$w.json" $w
done
