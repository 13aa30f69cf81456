#!/bin/bash
# stock-torch ResNet-18 reference (channels_last and NCHW) + rocprofv3 kernel stats of ours
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python benchmarks/torch_reference_resnet.py --steps 10 --warmup 5 > gpurun_out/torch_resnet_cl.log 2>&1 || exit $?
timeout -k 10 500 python benchmarks/torch_reference_resnet.py --steps 10 --warmup 5 --no-channels-last > gpurun_out/torch_resnet_nchw.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_resnet.log 2>&1
rc=$?
tail -3 gpurun_out/torch_resnet_cl.log gpurun_out/torch_resnet_nchw.log gpurun_out/prof_resnet.log
exit $rc
