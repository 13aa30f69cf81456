#!/bin/bash
# Round-3 pass X: c_proj dgrad on the K-major weight image + deferred column sums - tests, then
# GPT-2 bench A/B (default vs RTDC_DGRAD_KMAJOR=0 vs RTDC_COLSUM_DEFER=0, two rounds).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_wgrad_group_gpu.py tests/test_gpt2_parity_gpu.py tests/test_optim_overlap_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/x_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/x_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base RTDC_DGRAD_KMAJOR=0 RTDC_COLSUM_DEFER=0; do
    e=$([ $v = base ] && echo "" || echo "$v")
    env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_x_${v}_r$r.log 2>&1
    rc=$?; echo "GPT2 $v r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_x_${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
