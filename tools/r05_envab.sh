#!/bin/bash
# GPU box: A/B of env-step kernel builds on one box (envstep sub-bench, HIP-graph replay), alternating.
# usage: bash tools/r05_envab.sh <tag> <lib suffix> [<lib suffix> ...]   ("" = the product libecohip.so)
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1}"; shift
mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in "$@"; do
    lib="$ROOT/eco-dqn_amd/eco_hip/libecohip${v:+_$v}.so"
    ECO_HIP_LIB="$lib" timeout -k 10 120 python -u bench.py --workload envstep --steps 200 --warmup 20 \
      > "$OUT/envstep_${v:-product}_$rep.json" 2> "$OUT/envstep_${v:-product}_$rep.err" || { tail -3 "$OUT/envstep_${v:-product}_$rep.err"; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['roofline']['avg_launch_ms']*1e3,2), 'us')" "$OUT/envstep_${v:-product}_$rep.json" "${v:-product}" $rep
  done
done
