#!/bin/bash
# A/B of the weight-gradient reduction (bf16x3 default vs ECO_WGRAD_F32=1) on the train bench,
# with rocprofv3 kernel stats per variant.  Run on the GPU box via gpurun.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_wgrad
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/bf3" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_bf3.json"
ECO_WGRAD_F32=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/f32" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_f32.json"
echo done
