#!/bin/bash
# Round-3 pass W: c_proj dgrad on the K-major weight image (persistent kernel) - tests, then
# GPT-2 bench A/B (RTDC_DGRAD_KMAJOR=1 vs 0, alternating, two rounds).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "transposed or kmajor or fused_mlp" tests/test_gpt2_parity_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/kmajor_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/kmajor_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    RTDC_DGRAD_KMAJOR=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_kmaj${v}_r$r.log 2>&1
    rc=$?; echo "GPT2 KMAJOR=$v r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_kmaj${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
