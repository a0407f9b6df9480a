#!/bin/bash
# GPU box: interleaved train-bench A/B of the weight-gradient staging pipeline -- register buffers in flight
# (WGRAD_DEPTH 2 / 3 / 4) and nontemporal loads (WGRAD_NT) -- variant libraries from `make tvariant`.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab4"
L=$ROOT/eco-dqn_amd/eco_hip
for v in def nt d3 d3nt d4 def2 nt2 d32 d3nt2 d42; do
  case $v in
    def|def2) e="";; *) e="ECO_HIP_LIB=$L/libecohip_${v%2}.so";;
  esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab4/$v.json" 2>"$ROOT/gpurun_out/ab4/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab4/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
