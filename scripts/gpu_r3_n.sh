#!/bin/bash
# Round-3 pass N: implicit-GEMM convolutions with 3 / 4 LDS stages (RTDC_CONV_NS) - CNN GPU tests
# under each setting, then ResNet-18 benches interleaved 2,3,4,2,3,4.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for ns in 3 4; do
  RTDC_CONV_NS=$ns timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cnn_tests_ns$ns.log 2>&1
  rc=$?; echo "CNN TESTS NS=$ns EXIT $rc"; tail -n 3 gpurun_out/cnn_tests_ns$ns.log
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for ns in 2 3 4; do
    RTDC_CONV_NS=$ns timeout -k 10 200 python bench.py --model resnet18 --steps 20 --warmup 5 --no-ckpt > gpurun_out/resnet_ns${ns}_r$r.log 2>&1
    rc=$?; echo "RESNET NS=$ns r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_ns${ns}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
