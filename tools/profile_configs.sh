#!/bin/bash
# rocprofv3 kernel statistics of the non-default bench configurations (run on the GPU box via gpurun):
#   BA-500 train (configs[3] single-GPU leg), G22-like inference (configs[4]), ER-20 inference (configs[1])
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_configs
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/ba500" -o run -- \
  python3 "$ROOT/bench.py" --graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/ba500.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/gset" -o run -- \
  python3 "$ROOT/bench.py" --workload gset --steps 20 --warmup 3 > "$OUT/gset.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/er20" -o run -- \
  python3 "$ROOT/bench.py" --workload er20 --steps 40 --warmup 5 > "$OUT/er20.json"
echo "profile passes done: $OUT"
