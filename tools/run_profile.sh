#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun):
#   1) kernel trace + stats  2) FETCH_SIZE  3) WRITE_SIZE   (separate PMC passes,
#   MI355X_MICROARCH.md "HBM": FETCH_SIZE reads 1/2 of wide streaming reads on gfx950)
# usage: bash tools/run_profile.sh <tag> [bench args...]
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
shift || true
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/bench_trace.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench_fetch.json"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench_write.json"
echo "profile passes done: $OUT"
