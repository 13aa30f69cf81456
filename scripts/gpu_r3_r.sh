#!/bin/bash
# Round-3 pass Q: N <= 64 implicit-GEMM convolutions on 8-wave 256x64 tiles (RTDC_CONV64_W8) -
# CNN GPU tests under it, then ResNet-18 benches interleaved W8=1,0,1,0.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
RTDC_CONV128_W8=1 timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cnn_tests_w8_128.log 2>&1
rc=$?; echo "CNN TESTS W8 EXIT $rc"; tail -n 3 gpurun_out/cnn_tests_w8_128.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for w in 1 0; do
    RTDC_CONV128_W8=$w timeout -k 10 200 python bench.py --model resnet18 --steps 20 --warmup 5 --no-ckpt > gpurun_out/resnet_w8_128_${w}_r$r.log 2>&1
    rc=$?; echo "RESNET W8=$w r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_w8_128_${w}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
RTDC_CONV128_W8=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet_w8_128 -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_resnet_w8_128.log 2>&1
rc=$?; echo "PROF EXIT $rc"
[ $rc -eq 0 ] || exit $rc
t=$(find gpurun_out/prof_resnet_w8_128 -name '*kernel_trace.csv' | head -1)
python3 scripts/kstep.py "$t" --marker sgd_kernel > gpurun_out/prof_resnet_w8_128_step.txt
grep "128, 128" gpurun_out/prof_resnet_w8_128_step.txt | head -20
