#!/bin/bash
# Round-3 pass LL: tiled conv weight flip + split BatchNorm-statistics merge - CNN GPU tests,
# then ResNet-18 A/B of RTDC_BN_SPLIT_FINALIZE (alternating, two rounds).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/ll_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/ll_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    RTDC_BN_SPLIT_FINALIZE=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_ll_split${v}_r$r.log 2>&1
    rc=$?; echo "RESNET BN_SPLIT_FINALIZE=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_ll_split${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
