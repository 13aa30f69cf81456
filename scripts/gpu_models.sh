#!/bin/bash
# BASELINE configs 2 and 4 on one GPU: ResNet-18 (with the checkpoint phase) and Llama-3-8B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_cnn.log 2>&1
rc=$?; echo "CNN TESTS EXIT $rc"; tail -n 2 gpurun_out/t_cnn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/bench_resnet.log 2>&1
rc=$?; echo "RESNET EXIT $rc"; tail -n 1 gpurun_out/bench_resnet.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --model llama3-8b --steps 4 --warmup 2 --no-ckpt > gpurun_out/bench_llama.log 2>&1
rc=$?; echo "LLAMA EXIT $rc"; tail -n 1 gpurun_out/bench_llama.log
