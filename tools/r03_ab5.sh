#!/bin/bash
# GPU box: interleaved train-bench A/B of the replay sample's workgroup size (ECO_SAMPLE_THREADS 256 / 128 / 64),
# then the kernel trace of each (rocprofv3 --kernel-trace --stats, replay_compact_sample_kernel's duration).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab5"
for v in ${AB5_BENCH-256 128 64 256b 128b 64b}; do
  ECO_SAMPLE_THREADS=${v%b} timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab5/t$v.json" 2>"$ROOT/gpurun_out/ab5/t$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab5/t$v.json').read().strip().splitlines()[-1]); print('t$v', round(d['value']), round(d['ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp
for v in 256 128 64; do
  ECO_SAMPLE_THREADS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/ab5/prof_$v" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 6
  f=$(find "$ROOT/gpurun_out/ab5/prof_$v" -name "*kernel_stats.csv" | head -1)
  echo "t$v $(grep -E 'replay_compact_sample' "$f" | cut -d, -f1-4)"
done
