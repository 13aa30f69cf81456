#!/bin/bash
# Round-3 pass DD: kernel traces of this build - GPT-2-small and ResNet-18 benches under
# rocprofv3 (kernel stats + per-step kernel sequence), then plain benches of both (3 runs each).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_prof_gpt2.sh > gpurun_out/dd_prof_gpt2.out 2>&1
rc=$?; echo "PROF GPT2 EXIT $rc"; head -3 gpurun_out/prof_gpt2_summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --no-ckpt > gpurun_out/prof_resnet.log 2>&1
rc=$?; echo "PROF RESNET EXIT $rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_resnet -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 13 40 > gpurun_out/prof_resnet_summary.txt
t=$(find gpurun_out/prof_resnet -name '*kernel_trace.csv' | head -1)
python3 scripts/kstep.py "$t" > gpurun_out/prof_resnet_step.txt
head -3 gpurun_out/prof_resnet_summary.txt
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/dd_gpt2_r$r.log 2>&1
  rc=$?; echo "GPT2 r$r EXIT $rc $(tail -n 1 gpurun_out/dd_gpt2_r$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/dd_resnet_r$r.log 2>&1
  rc=$?; echo "RESNET r$r EXIT $rc $(tail -n 1 gpurun_out/dd_resnet_r$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
