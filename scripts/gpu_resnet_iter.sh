#!/bin/bash
# ResNet iteration: conv/BN numerics, bench, kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_cnn_gpu.py tests/test_kernels_gpu.py -x -q > gpurun_out/cnn_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 30 gpurun_out/cnn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/bench_resnet.log 2>&1
rc=$?; echo "RESNET EXIT $rc"; tail -n 2 gpurun_out/bench_resnet.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_resnet.log 2>&1
echo "PROF EXIT $?"
