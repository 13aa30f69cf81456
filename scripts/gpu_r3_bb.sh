#!/bin/bash
# Round-3 pass BB: BatchNorm-backward statistics in the stride-1 dgrad epilogue (conv_gemm_bnb) -
# CNN GPU tests, then ResNet-18 A/B (RTDC_BNB_FUSED=1 vs 0, alternating, two rounds).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_models_gpu.py tests/test_optim_overlap_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/bb_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/bb_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    RTDC_BNB_FUSED=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_bb_${v}_r$r.log 2>&1
    rc=$?; echo "RESNET BNB_FUSED=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_bb_${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
