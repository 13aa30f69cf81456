#!/bin/bash
# Round-3 pass J: ResNet-18 bench + kernel trace with the per-step kernel sequence (per-conv
# times, to place the 8-wave implicit-GEMM kernel), GPT-2 bench (unprofiled, this build).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --no-ckpt > gpurun_out/bench_resnet.log 2>&1
rc=$?; echo "RESNET EXIT $rc"; tail -n 1 gpurun_out/bench_resnet.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo "GPT2 EXIT $rc"; tail -n 1 gpurun_out/bench_gpt2.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_resnet.log 2>&1
rc=$?; echo "PROF EXIT $rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_resnet -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 7 40 > gpurun_out/prof_resnet_summary.txt
t=$(find gpurun_out/prof_resnet -name '*kernel_trace.csv' | head -1)
python3 scripts/kstep.py "$t" --marker sgd_kernel > gpurun_out/prof_resnet_step.txt
head -30 gpurun_out/prof_resnet_summary.txt
