#!/bin/bash
# GPU box: train-bench A/B of the weight-gradient split after the narrow-X change (ECO_WGRAD_BIG = workgroups per
# K = 128 job, the rest by rows), interleaved.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab2"
for v in def big96 big72 big104 def2 big96b; do
  case $v in def|def2) e="";; big96|big96b) e="ECO_WGRAD_BIG=96";; big72) e="ECO_WGRAD_BIG=72";; big104) e="ECO_WGRAD_BIG=104";; esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab2/$v.json" 2>"$ROOT/gpurun_out/ab2/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab2/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
