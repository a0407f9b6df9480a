#!/bin/bash
# GPU box: the dense kernels for 224 < N <= 512 (eco_mpnn_dl.h): parity tests, BA-500 bench, phase timing.
mkdir -p gpurun_out/dl
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_dense_gpu.py::test_dense_large_matches_csr_and_oracle "tests/test_mpnn_gpu.py::test_forward_matches_oracle_at_scale" \
  tests/test_parity_bench_sizes_gpu.py::test_backward_ba500_m2048_matches_autograd \
  "tests/test_parity_bench_sizes_gpu.py::test_shared_graph_forward_matches_per_episode_and_oracle" \
  tests/test_parity_bench_sizes_gpu.py::test_shared_graph_forward_hub_and_isolated_nodes \
  tests/test_parity_benched_batches_gpu.py > gpurun_out/dl/tests.log 2>&1
rc=$?; tail -5 gpurun_out/dl/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --graph BA --n 500 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/dl/ba500.json 2> gpurun_out/dl/ba500.err || exit 5
python3 -c "import json; d=json.loads(open('gpurun_out/dl/ba500.json').read().strip().splitlines()[-1]); print('ba500', round(d['value']), 'ms/step', round(d['ms_per_step'],3), d.get('kernels_ms_per_step'))"
timeout -k 10 300 python -u tools/phase_timing.py --n 500 --graph BA --p 4 > gpurun_out/dl/phase_ba500.txt 2>&1 || exit 6
cat gpurun_out/dl/phase_ba500.txt
timeout -k 10 300 python -u bench.py --workload gset --steps 20 --warmup 3 > gpurun_out/dl/gset.json 2> gpurun_out/dl/gset.err || exit 7
python3 -c "import json; d=json.loads(open('gpurun_out/dl/gset.json').read().strip().splitlines()[-1]); print('gset', round(d['value']), 'ms/step', round(d['ms_per_step'],3))"
