#!/bin/bash
# GPU box: tests/test_split2_hazard_gpu.py and the cross-path bitwise tests that failed in round 4 without the
# v_fma_mix wait states, on the product library and then on the negative-control build
# (make -C eco-dqn_amd variant V=split2neg XFLAGS=-DECO_SPLIT2_NEGATIVE_CONTROL, built in the container).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/${1:-r06_split2}"
mkdir -p "$OUT"
SEL="tests/test_split2_hazard_gpu.py"
timeout -k 10 300 python -u -m pytest $SEL -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/product.log" 2>&1
echo "product rc=$?"; grep -E "passed|failed" "$OUT/product.log" | tail -2
ECO_HIP_LIB="$ROOT/eco-dqn_amd/eco_hip/libecohip_split2neg.so" timeout -k 10 300 python -u -m pytest $SEL -m gpu -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/negative_control.log" 2>&1
echo "negative control rc=$? (expected: failed)"; grep -E "FAILED|passed|failed" "$OUT/negative_control.log" | tail -8
exit 0
