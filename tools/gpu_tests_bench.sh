#!/bin/bash
# GPU box: the -m gpu suite (one process) then, unless it faulted / hung / aborted, one bench run.
# usage: tools/gpu_tests_bench.sh [pytest selection...]
mkdir -p gpurun_out
sel="${@:-tests}"
timeout -k 10 1000 python -u -m pytest $sel -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gputests.log 2>&1
rc=$?
tail -5 gpurun_out/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json
exit $(( rc > brc ? rc : brc ))
