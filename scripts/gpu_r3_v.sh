#!/bin/bash
# Round-3 pass V (re-entry): full GPU test suite on the rebuilt extension, then the ResNet-18
# product path (trainer + async DCP every 50 steps, exact resume, uninterrupted run, bench).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_full_v.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/tests_full_v.log
[ $rc -eq 0 ] || exit $rc
MODEL=resnet18 OUT=gpurun_out/product_resnet_r3 bash scripts/gpu_product_r3.sh
