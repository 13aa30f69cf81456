#!/bin/bash
# GPT-2-small headline bench (with checkpoint phase) + kernel-time profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/bench_gpt2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_gpt2.log 2>&1
echo "PROF EXIT $?"
