#!/bin/bash
# Round-3 pass PP: 128- vs 64-pixel chunks of the 3x3 weight-gradient kernel.
# tests, ResNet-18 parity, then a ResNet-18 A/B of RTDC_CONV3_WGRAD and a kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
RTDC_CONV3_KP=128 timeout -k 10 400 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pp_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 15 gpurun_out/pp_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 128 64; do
    RTDC_CONV3_KP=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_pp_kp${v}_r$r.log 2>&1
    rc=$?; echo "RESNET CONV3_KP=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_pp_kp${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_prof -o run -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --no-ckpt > gpurun_out/pp_prof.log 2>&1
rc=$?; echo "PROF EXIT $rc"
f=$(find gpurun_out/pp_prof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -14 "$f" | cut -c1-160
exit $rc
