#!/bin/bash
# GPU box: configs[3] (BA-500 x 8192 train loop) A/B of the DL kernels with 8 waves x 4 tiles (default) and
# 16 waves x 2 tiles (libecohip_dl16.so, DL_NW_X=16), interleaved.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/dl16"
for v in def dl16 def2 dl162; do
  case $v in def|def2) e="";; dl16|dl162) e="ECO_HIP_LIB=$ROOT/eco-dqn_amd/eco_hip/libecohip_dl16.so";; esac
  env $e timeout -k 10 300 python -u bench.py --graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/dl16/$v.json" 2>"$ROOT/gpurun_out/dl16/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/dl16/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
