#!/bin/bash
# rocprofv3 kernel stats of the configs[4] bench (gset) on the GPU box
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_gset
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --workload gset --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
head -12 "$OUT/trace/run_kernel_stats.csv" | cut -c1-220
exit $rc
