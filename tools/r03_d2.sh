#!/bin/bash
# GPU box: dense2 (fp16x2) forward -- parity tests, then A/B bench against the bf16x3 kernel.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mpnn_gpu.py tests/test_dense_gpu.py tests/test_parity_benched_batches_gpu.py \
  tests/test_parity_bench_sizes_gpu.py tests/test_dqn_gpu.py tests/test_problems_train_gpu.py tests/test_parallel_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/d2_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/d2_tests.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/d2_bench.json 2> gpurun_out/d2_bench.err || exit 3
ECO_DENSE_V1=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/d1_bench.json 2> gpurun_out/d1_bench.err || exit 3
python - <<'PY'
import json
for f in ("d2", "d1"):
    d = json.loads(open(f"gpurun_out/{f}_bench.json").read().strip().splitlines()[-1])
    print(f, round(d["value"]), "ms/step", round(d["ms_per_step"], 2), d["kernels_ms_per_step"], "fwd avg ms", round(d["roofline"]["avg_launch_ms"], 4))
PY
exit $rc
