#!/bin/bash
# Round-3 pass II: kernel trace of the Llama-3-8B one-GPU bench (this build) + BN statistics grid A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o run -- python3 bench.py --model llama3-8b --steps 4 --warmup 2 --no-ckpt > gpurun_out/prof_llama.log 2>&1
rc=$?; echo "PROF LLAMA EXIT $rc"; tail -n 1 gpurun_out/prof_llama.log | grep -o '"ms_per_step": [0-9.]*'
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_llama -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 6 40 > gpurun_out/prof_llama_summary.txt
t=$(find gpurun_out/prof_llama -name '*kernel_trace.csv' | head -1)
python3 scripts/kstep.py "$t" > gpurun_out/prof_llama_step.txt
head -30 gpurun_out/prof_llama_summary.txt
bash scripts/gpu_r3_hh.sh
