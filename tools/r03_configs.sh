#!/bin/bash
# GPU box: the non-default bench configurations with kernel stats: BA-500 train (configs[3] single-GPU leg),
# G22-like (configs[4]), ER-20 (configs[1]); plus BA-500 phase timing.
mkdir -p gpurun_out/pc
ROOT=$(pwd)
timeout -k 10 300 python -u tools/phase_timing.py --n 500 --graph BA --p 4 > gpurun_out/pc/phase_ba500.txt 2>&1 || { echo "phase rc=$?"; tail -3 gpurun_out/pc/phase_ba500.txt; exit 3; }
cd /tmp && export TMPDIR=/tmp
for w in ba500 gset er20; do
  case $w in
    ba500) args="--graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline";;
    gset) args="--workload gset --steps 20 --warmup 3";;
    er20) args="--workload er20 --steps 40 --warmup 5";;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $ROOT/gpurun_out/pc/$w -o run -- \
    python3 $ROOT/bench.py $args > $ROOT/gpurun_out/pc/$w.json || exit 4
  python3 -c "import json; d=json.loads(open('$ROOT/gpurun_out/pc/$w.json').read().strip().splitlines()[-1]); print('$w', round(d['value']), 'ms/step', round(d['ms_per_step'],3))"
  head -8 $ROOT/gpurun_out/pc/$w/run_kernel_stats.csv | cut -d, -f1-4
done
