#!/bin/bash
# Round-3 pass Z: deferred column sums restricted to flat-buffer slots + fused stem pool/BN
# backward - affected GPU tests, then ResNet-18 A/B (RTDC_POOL_BN_FUSED) and GPT-2 A/B
# (RTDC_COLSUM_DEFER), two rounds each.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wgrad_group_gpu.py tests/test_optim_overlap_gpu.py tests/test_cnn_gpu.py tests/test_gpt2_parity_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/z_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/z_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    RTDC_POOL_BN_FUSED=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_z_pool${v}_r$r.log 2>&1
    rc=$?; echo "RESNET POOL_BN_FUSED=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_z_pool${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
  for v in 1 0; do
    RTDC_COLSUM_DEFER=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_z_defer${v}_r$r.log 2>&1
    rc=$?; echo "GPT2 COLSUM_DEFER=$v r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_z_defer${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
