#!/bin/bash
# GPU box: selected -m gpu tests in one process, then one bench workload, each under its own time limit.
# usage: tools/gpu_quick.sh "<pytest files>" "<bench args>"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $1 -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/quick_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/quick_tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -n "$2" ]; then
  timeout -k 10 400 python -u bench.py $2 > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
  brc=$?
  cat gpurun_out/quick_bench.json
  [ $brc -ne 0 ] && tail -20 gpurun_out/quick_bench.err
  exit $(( rc > brc ? rc : brc ))
fi
exit $rc
