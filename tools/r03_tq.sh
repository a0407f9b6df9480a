#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_training_quality_gpu.py tests/test_dqn_gpu.py tests/test_parallel_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tq_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error|mean best" gpurun_out/tq_tests.log | tail -30
exit $rc
