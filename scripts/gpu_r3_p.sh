#!/bin/bash
# Round-3 pass P: grouped weight gradients on a side stream (RTDC_WGRAD_SIDE) - group tests under
# it, then GPT-2 benches interleaved SIDE=1,0,1,0.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
RTDC_WGRAD_SIDE=1 timeout -k 10 400 python -u -m pytest tests/test_wgrad_group_gpu.py tests/test_optim_overlap_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/wgrad_side_tests.log 2>&1
rc=$?; echo "SIDE TESTS EXIT $rc"; tail -n 4 gpurun_out/wgrad_side_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for g in 1 0; do
    RTDC_WGRAD_SIDE=$g timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_side${g}_r$r.log 2>&1
    rc=$?; echo "GPT2 SIDE=$g r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_side${g}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
