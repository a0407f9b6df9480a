#!/bin/bash
# GPU box: the swizzled weight-gradient LDS layout (libecohip_swz.so, WGRAD_SWZ=1: 37 KB per workgroup, 4 per CU):
# backward / train-step parity tests on it, interleaved train-bench A/B, kernel durations under rocprofv3.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/ab8"
L=$ROOT/eco-dqn_amd/eco_hip
ECO_HIP_LIB=$L/libecohip_swz.so timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_dqn_gpu.py \
  tests/test_parity_bench_sizes_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$ROOT/gpurun_out/ab8/tests.log" 2>&1
rc=$?; tail -3 "$ROOT/gpurun_out/ab8/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in def swz def2 swz2; do
  case $v in def|def2) e="";; *) e="ECO_HIP_LIB=$L/libecohip_swz.so";; esac
  env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/ab8/$v.json" 2>"$ROOT/gpurun_out/ab8/$v.err" || exit 5
  python3 -c "import json,sys; d=json.loads(open('$ROOT/gpurun_out/ab8/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
done
cd /tmp && export TMPDIR=/tmp
for v in def swz; do
  case $v in def) lib=$L/libecohip.so;; *) lib=$L/libecohip_swz.so;; esac
  ECO_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/ab8/prof_$v" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 6
  f=$(find "$ROOT/gpurun_out/ab8/prof_$v" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'wgrad' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0], r['Calls'], float(r['AverageNs']) / 1e3)
PY
done
