#!/bin/bash
# GPU box: the round-5 pins -- evaluation across ranks, quality (ER-200, BA-200), configs[3] at full size, the split2
# hazard probe and its negative control.  Each step under its own limit; stops at the first failure.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r05val}"
mkdir -p "$OUT"
run() {  # name, timeout, pytest args
  timeout -k 10 $2 python -u -m pytest $3 -m gpu -x -v -s --timeout $2 --timeout-method thread -p no:cacheprovider \
    > "$OUT/$1.log" 2>&1
  local rc=$?
  echo "$1 rc=$rc"; grep -E "ratio|EVAL_OK|configs\[3\]|passed|failed|Error" "$OUT/$1.log" | tail -8
  return $rc
}
run eval 400 "tests/test_parallel_gpu.py" || exit 1
run split2 120 "tests/test_split2_hazard_gpu.py" || exit 2
ECO_HIP_LIB="$ROOT/eco-dqn_amd/eco_hip/libecohip_split2neg.so" timeout -k 10 120 python -u -m pytest \
  tests/test_split2_hazard_gpu.py -m gpu -v --timeout 60 --timeout-method thread -p no:cacheprovider \
  > "$OUT/split2_negative_control.log" 2>&1
echo "negative control rc=$? (expected: failed)"; grep -E "passed|failed|differ" "$OUT/split2_negative_control.log" | tail -3
run configs3 600 "tests/test_configs3_fullsize_gpu.py" || exit 3
run quality_er200 900 "tests/test_training_quality_er200_gpu.py" || exit 4
run quality_ba200 900 "tests/test_training_quality_ba200_gpu.py" || exit 5
