#!/bin/bash
# GPU box: kernel trace of the configs[2] train bench + per-phase timing of the dense kernels (M=2048 ER-200).
mkdir -p gpurun_out/p3
ROOT=$(pwd)
timeout -k 10 300 python -u tools/phase_timing.py > gpurun_out/p3/phase_timing.txt 2>&1 || { echo "phase timing rc=$?"; tail gpurun_out/p3/phase_timing.txt; exit 3; }
cat gpurun_out/p3/phase_timing.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $ROOT/gpurun_out/p3/train -o run -- \
  python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $ROOT/gpurun_out/p3/train.json || exit 4
head -12 $(find $ROOT/gpurun_out/p3/train -name "*kernel_stats.csv" | head -1) | cut -d, -f1-8
