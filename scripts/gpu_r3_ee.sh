#!/bin/bash
# Round-3 pass EE: branch-free stem pool gather (4 windows loaded together, 2 positions per
# iteration) - CNN tests, ResNet-18 A/B (RTDC_POOL_BN_FUSED), kernel stats of the stem kernels.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/ee_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/ee_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    RTDC_POOL_BN_FUSED=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_ee_${v}_r$r.log 2>&1
    rc=$?; echo "RESNET POOL_BN_FUSED=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_ee_${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet_ee -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_resnet_ee.log 2>&1
rc=$?; echo "PROF EXIT $rc"
f=$(find gpurun_out/prof_resnet_ee -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 8 40 > gpurun_out/prof_resnet_ee_summary.txt
grep -i "pool\|maxpool" gpurun_out/prof_resnet_ee_summary.txt
