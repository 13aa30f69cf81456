#!/bin/bash
# Kernel trace of the GPT-2-small bench: per-kernel stats + timeline gaps
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python3 bench.py --steps 10 --warmup 3 --no-ckpt "$@" > gpurun_out/prof_gpt2.log 2>&1
rc=$?; echo "PROF EXIT $rc"; tail -n 2 gpurun_out/prof_gpt2.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_gpt2 -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 13 40 > gpurun_out/prof_gpt2_summary.txt
t=$(find gpurun_out/prof_gpt2 -name '*kernel_trace.csv' | head -1)
python3 scripts/ktimeline.py "$t" --last-ms 100 >> gpurun_out/prof_gpt2_summary.txt
cat gpurun_out/prof_gpt2_summary.txt | head -80
python3 scripts/kstep.py "$t" > gpurun_out/prof_gpt2_step.txt
