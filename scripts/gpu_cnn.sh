#!/bin/bash
# ResNet-18 / Llama kernels + model numerics, then the ResNet-18 and Llama-1B benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_cnn_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/cnn_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -30 gpurun_out/cnn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/bench_resnet.log 2>&1
rc=$?; echo "RESNET EXIT $rc"; tail -5 gpurun_out/bench_resnet.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model llama3-1b --steps 5 --warmup 2 > gpurun_out/bench_llama1b.log 2>&1
rc=$?; echo "LLAMA EXIT $rc"; tail -5 gpurun_out/bench_llama1b.log
exit $rc
