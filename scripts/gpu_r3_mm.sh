#!/bin/bash
# Round-3 pass MM: 3x3/s1 conv weight gradient with input reuse (conv3x3_wgrad_kernel) - conv
# tests, ResNet-18 parity, then a ResNet-18 A/B of RTDC_CONV3_WGRAD and a kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/mm_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 15 gpurun_out/mm_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    RTDC_CONV3_WGRAD=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_mm_w3${v}_r$r.log 2>&1
    rc=$?; echo "RESNET CONV3_WGRAD=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_mm_w3${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/mm_prof -o run -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --no-ckpt > gpurun_out/mm_prof.log 2>&1
rc=$?; echo "PROF EXIT $rc"
f=$(find gpurun_out/mm_prof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -14 "$f" | cut -c1-160
exit $rc
