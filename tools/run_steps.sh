#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop after a step that faulted, aborted, hung or
# was killed (exit status other than 0 / 1).   usage: tools/run_steps.sh <seconds> '<cmd>' [<seconds> '<cmd>' ...]
mkdir -p gpurun_out
i=0
while [ $# -ge 2 ]; do
  t=$1; c=$2; shift 2; i=$((i+1))
  echo "== step $i: $c"
  timeout -k 10 "$t" bash -c "$c"
  rc=$?
  echo "== step $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
