#!/bin/bash
# GPU box: interleaved train-bench A/B of the weight-gradient grid: 2 / 3 (default) / 4 workgroups per CU
# (WGRAD_WG_X; 46 KB of LDS each, so 3 are resident), then each under rocprofv3 for the kernel's duration.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab7"
L=$ROOT/eco-dqn_amd/eco_hip
for v in def wg2 wg4 def2 wg22 wg42; do
  case $v in def|def2) e="";; *) e="ECO_HIP_LIB=$L/libecohip_${v:0:3}.so";; esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab7/$v.json" 2>"$ROOT/gpurun_out/ab7/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab7/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
cd /tmp && export TMPDIR=/tmp
for v in def wg2 wg4; do
  case $v in def) lib=$L/libecohip.so;; *) lib=$L/libecohip_$v.so;; esac
  ECO_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/ab7/prof_$v" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 6
  f=$(find "$ROOT/gpurun_out/ab7/prof_$v" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'wgrad' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0], r['Calls'], float(r['AverageNs']) / 1e3)
PY
done
