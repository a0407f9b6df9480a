#!/bin/bash
# GPU box, round 3: new parity tests, then training-quality probes (each step under its own limit).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_benched_batches_gpu.py tests/test_dqn_gpu.py -k "b1024 or b4096 or quirk or regenerate" \
  -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r03_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 420 python -u tools/train_er20.py --envs 64 --minibatch 64 --steps 600000 --eval-every 50000 \
  --out gpurun_out/q_b64_m64.json > gpurun_out/q_b64_m64.log 2>&1 || { echo "probe1 rc=$?"; tail -5 gpurun_out/q_b64_m64.log; exit 3; }
tail -3 gpurun_out/q_b64_m64.log
timeout -k 10 420 python -u tools/train_er20.py --envs 2048 --minibatch 512 --steps 1000000 --eval-every 100000 \
  --out gpurun_out/q_b2048_m512.json > gpurun_out/q_b2048_m512.log 2>&1 || { echo "probe2 rc=$?"; tail -5 gpurun_out/q_b2048_m512.log; exit 3; }
tail -3 gpurun_out/q_b2048_m512.log
exit $rc
