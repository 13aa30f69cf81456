#!/bin/bash
# Round-3 pass M: kernel trace of the 1-rank RCCL (--force-dist) GPT-2 step: what DDP adds
# per step over the plain 1-GPU step (RCCL kernels, copies, stream waits).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ddp1 -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --force-dist --no-ckpt --sweep 0 > gpurun_out/prof_ddp1.log 2>&1
rc=$?; echo "PROF EXIT $rc"; tail -n 1 gpurun_out/prof_ddp1.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_ddp1 -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 13 40 > gpurun_out/prof_ddp1_summary.txt
t=$(find gpurun_out/prof_ddp1 -name '*kernel_trace.csv' | head -1)
python3 scripts/ktimeline.py "$t" --last-ms 100 >> gpurun_out/prof_ddp1_summary.txt
python3 scripts/kstep.py "$t" > gpurun_out/prof_ddp1_step.txt
head -60 gpurun_out/prof_ddp1_summary.txt
tail -3 gpurun_out/prof_ddp1_step.txt
