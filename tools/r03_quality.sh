#!/bin/bash
# GPU box: large-batch training-quality sweep on ER-20 (tools/train_er20.py), each run under its own limit.
mkdir -p gpurun_out/q
run() { tag=$1; shift; timeout -k 10 300 python -u tools/train_er20.py "$@" --out gpurun_out/q/$tag.json > gpurun_out/q/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 gpurun_out/q/$tag.log; exit 3; }; python -c "import json; d=json.load(open('gpurun_out/q/$tag.json')); print('$tag', d['grad_steps'], [round(c[1],3) for c in d['curve']], d['final_50attempts'])"; }
run b2048_m512_lr1e4_gs --envs 2048 --minibatch 512 --lr 1e-4 --steps 1000000 --eval-every 100000
run b2048_m512_lr3e4_gs --envs 2048 --minibatch 512 --lr 3e-4 --steps 1000000 --eval-every 100000
run b2048_m512_lr3e4_smp --envs 2048 --minibatch 512 --lr 3e-4 --steps 1000000 --eval-every 100000 --target-sync samples
run b2048_m512_lr1e3_gs --envs 2048 --minibatch 512 --lr 1e-3 --steps 1000000 --eval-every 100000
run b64_m64_gs --envs 64 --minibatch 64 --lr 1e-4 --steps 400000 --eval-every 50000
