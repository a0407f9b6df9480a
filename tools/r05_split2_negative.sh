#!/bin/bash
# GPU box: tests/test_split2_hazard_gpu.py on the product library, then on the negative-control build without the
# v_fma_mix wait states (make variant V=split2neg XFLAGS=-DECO_SPLIT2_NEGATIVE_CONTROL, built in the container).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r05_split2}"
mkdir -p "$OUT"
timeout -k 10 120 python -u -m pytest tests/test_split2_hazard_gpu.py -m gpu -v --timeout 60 --timeout-method thread \
  -p no:cacheprovider > "$OUT/product.log" 2>&1
echo "product rc=$?"; grep -E "passed|failed" "$OUT/product.log" | tail -2
ECO_HIP_LIB="$ROOT/eco-dqn_amd/eco_hip/libecohip_split2neg.so" timeout -k 10 120 python -u -m pytest \
  tests/test_split2_hazard_gpu.py -m gpu -v --timeout 60 --timeout-method thread -p no:cacheprovider \
  > "$OUT/negative_control.log" 2>&1
echo "negative control rc=$? (expected: failed)"; grep -E "passed|failed|differ" "$OUT/negative_control.log" | tail -4
exit 0
