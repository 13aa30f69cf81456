#!/bin/bash
# Kernel trace of the ResNet-18 bench (256 x 224^2): per-kernel stats + timeline gaps
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --no-ckpt "$@" > gpurun_out/prof_resnet.log 2>&1
rc=$?; echo "PROF EXIT $rc"; tail -n 1 gpurun_out/prof_resnet.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_resnet -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 13 45 > gpurun_out/prof_resnet_summary.txt
t=$(find gpurun_out/prof_resnet -name '*kernel_trace.csv' | head -1)
python3 scripts/ktimeline.py "$t" --last-ms 60 >> gpurun_out/prof_resnet_summary.txt
