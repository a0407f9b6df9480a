#!/bin/bash
# GPU box: interleaved train-bench A/B -- the weight-gradient split (ECO_WGRAD_BIG) and the forward's Wf staged
# per wave (libecohip_wfw.so, D2_WF_PER_WAVE) -- then phase timing of the Wf-per-wave forward.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab3"
W=$ROOT/eco-dqn_amd/eco_hip/libecohip_wfw.so
for v in def wfw big96 big72 def2 wfw2 big104; do
  case $v in
    def|def2) e="";; wfw|wfw2) e="ECO_HIP_LIB=$W";; big96) e="ECO_WGRAD_BIG=96";; big72) e="ECO_WGRAD_BIG=72";;
    big104) e="ECO_WGRAD_BIG=104";;
  esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab3/$v.json" 2>"$ROOT/gpurun_out/ab3/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab3/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
ECO_HIP_LIB=$ROOT/eco-dqn_amd/eco_hip/libecohip_wfwt.so timeout -k 10 300 python -u tools/phase_timing.py > "$ROOT/gpurun_out/ab3/phase_wfw.txt" 2>&1 || exit 6
head -12 "$ROOT/gpurun_out/ab3/phase_wfw.txt"
