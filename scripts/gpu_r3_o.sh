#!/bin/bash
# Round-3 pass O: grouped weight gradients - new GPU tests, the full GPU suite, then GPT-2 benches
# interleaved RTDC_WGRAD_GROUP=1,0,1,0 and a kernel trace of the grouped step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wgrad_group_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/wgrad_group_tests.log 2>&1
rc=$?; echo "GROUP TESTS EXIT $rc"; tail -n 8 gpurun_out/wgrad_group_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for g in 1 0; do
    RTDC_WGRAD_GROUP=$g timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_group${g}_r$r.log 2>&1
    rc=$?; echo "GPT2 GROUP=$g r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_group${g}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "ALL GPU TESTS EXIT $rc"; tail -n 5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_gpt2.sh > /dev/null 2>&1; echo "PROF EXIT $?"; head -25 gpurun_out/prof_gpt2_summary.txt
